#!/bin/bash
# nar1 iteration: narrow / headline parity, bench A/B (nar1 vs GW_NAR1=0), kernel-trace stats.
set -u
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_region_narrow.py tests/test_gpu_headline.py ${EXTRA_TESTS:-} -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/nar1_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r5/nar1_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/nar1_tests.log | head -20; exit $rc; fi
for v in default ${AB:-GW_NAR1=0}; do
  tag=${v//=/_}
  env $([ $v = default ] || echo $v) timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > gpurun_out/r5/bench_$tag.json 2> gpurun_out/r5/bench_$tag.err || { tail -20 gpurun_out/r5/bench_$tag.err; exit 4; }
  echo "$tag: $(python scripts/r5/jf.py gpurun_out/r5/bench_$tag.json value ms_per_step roofline.frac roofline.avg_launch_ms roofline.pass1_avg_ms roofline.apply_avg_ms)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/prof -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed > gpurun_out/r5/prof_bench.json 2> gpurun_out/r5/prof_bench.err || { tail -5 gpurun_out/r5/prof_bench.err; exit 5; }
f=$(ls gpurun_out/r5/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find gpurun_out/r5/prof -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.1f} total_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
