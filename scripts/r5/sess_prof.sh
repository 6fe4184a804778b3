#!/bin/bash
# Sessions config: kernel-trace stats of the slot sort path (hand-written sort).
set -u
mkdir -p gpurun_out/r5/sprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/sprof/prof -o run --output-format csv -- python -u scripts/configs_bench.py --only ${ONLY:-sessions} --steps ${STEPS:-20} --no-cpu-baseline > gpurun_out/r5/sprof/configs.jsonl 2> gpurun_out/r5/sprof/configs.err || { tail -5 gpurun_out/r5/sprof/configs.err; exit 5; }
f=$(find gpurun_out/r5/sprof/prof -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.1f} total_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
python scripts/r5/jf.py gpurun_out/r5/sprof/configs.jsonl value ms_per_step roofline.frac
