#!/bin/bash
# Session prep A/B: session + count-window parity suites, then the sessions and WindowWordCount
# config lines with the new library and flink_amd/libgpuwin_base.so, alternating.
# OUT: gpurun_out/r6/prep/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/prep
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_session_scenarios.py tests/test_gpu_session_groups.py tests/test_gpu_session_deferred.py tests/test_gpu_session_snapshot.py tests/test_gpu_count_windows.py tests/test_gpu_fullsize.py::test_sessions_avg_f64_12m_keys -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for tag in new base new2 base2; do
  case $tag in base*) export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_base.so;; *) unset GW_LIB_PATH;; esac
  timeout -k 10 400 python -u scripts/configs_bench.py --only sessions,wordcount --no-cpu-baseline > $O/cfg_$tag.jsonl 2> $O/cfg_$tag.err || { tail -20 $O/cfg_$tag.err; exit 4; }
  python -c "
import json
for l in open('$O/cfg_$tag.jsonl'):
    d=json.loads(l); print('$tag', d['config'].get('workload', d.get('metric'))[:20] if isinstance(d.get('config'),dict) else '', round(d['value']/1e9,3),'G',round(d['ms_per_step'],4),'ms')"
done
unset GW_LIB_PATH
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u scripts/configs_bench.py --only sessions --no-cpu-baseline > $O/prof.jsonl 2> $O/prof.err || { tail -5 $O/prof.err; exit 5; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_sessions.csv
