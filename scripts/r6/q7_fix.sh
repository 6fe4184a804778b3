#!/bin/bash
# The apply's staging with the mask reads issued beside the cell loads: parity suites that read
# retired cells, then Q7 and the headline against the build without the substitution (timing
# bound, results not checked).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6/q7fix
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_nar_carry.py tests/test_gpu_lateness.py tests/test_gpu_region_narrow.py tests/test_gpu_region_compact.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_window_classes.py tests/test_gpu_snapshot.py tests/test_gpu_restore.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for v in cur xnosub; do
  if [ ${v%2} = cur ]; then unset GW_LIB_PATH; else export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$v -o run --output-format csv -- python -u scripts/configs_bench.py --only q7 --no-cpu-baseline --steps 30 > $O/q7_$v.jsonl 2> $O/q7_$v.err || { echo "$v failed"; exit 4; }
  f=$(find $O/t_$v -name "*kernel_stats.csv" | head -1)
  echo "q7 $v $(python scripts/r5/jf.py $O/q7_$v.jsonl value) $(grep -E 'apply_nar' $f | awk -F, '{print $1, $3, $4}' | tr '\n' ' ')"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > $O/hl_$v.json 2> $O/hl_$v.err || { echo "$v hl failed"; exit 5; }
  echo "headline $v $(python scripts/r5/jf.py $O/hl_$v.json value roofline.frac roofline.apply_avg_ms)"
done
