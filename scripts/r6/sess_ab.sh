#!/bin/bash
# Sessions: the status zeroing by the one-wave kernel, session suites, then the config line
# against the previous build, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/sessab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_session_scenarios.py tests/test_gpu_session_groups.py tests/test_gpu_session_deferred.py tests/test_gpu_session_snapshot.py tests/test_gpu_count_windows.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in new base; do
    if [ $v = new ]; then unset GW_LIB_PATH; else export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_base.so; fi
    timeout -k 10 300 python -u scripts/configs_bench.py --only sessions --no-cpu-baseline --steps 40 > $O/s_${v}_$i.jsonl 2> $O/s_${v}_$i.err || { tail -5 $O/s_${v}_$i.err; exit 4; }
    echo "$v $i $(python scripts/r5/jf.py $O/s_${v}_$i.jsonl value ms_per_step)"
  done
done
