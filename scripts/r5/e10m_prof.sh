#!/bin/bash
# Q5 at E = 10M events per pane (1M-event batches): kernel trace over the bench.
set -u
O=gpurun_out/r5/e10m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python -u bench.py --events-per-pane 10000000 --no-host-fed --no-cpu-baseline ${EXTRA:-} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 5; }
python scripts/r5/jf.py $O/bench.json value ms_per_step roofline.frac roofline.avg_launch_ms roofline.fire_avg_launch_ms
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.1f} total_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
t=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python - "$t" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gw::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# time between consecutive P1 launches in the second half (steady state)
p1 = [int(r["Start_Timestamp"]) for r in rows if "k_rgn_p1" in r["Kernel_Name"]]
d = [(b - a) / 1e3 for a, b in zip(p1, p1[1:])]
h = d[len(d) // 2:]
print("P1-to-P1 us (second half): median", sorted(h)[len(h) // 2], "max", max(h))
PY
