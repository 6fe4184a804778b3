#!/bin/bash
# The exchange path at N = 1 (--force-exchange) under a kernel trace: per-kernel times and the
# per-step timeline (what separates consecutive P1 launches).
set -u
O=${XO:-gpurun_out/r5/xprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python -u bench.py --force-exchange --pack ${PACK:-auto} --no-host-fed --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 5; }
python scripts/r5/jf.py $O/bench.json value ms_per_step
f=$(find $O/trace -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.1f} total_ms={float(r["TotalDurationNs"])/1e6:8.2f}')
PY
t=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
p1 = [i for i, r in enumerate(rows) if "k_rgn_p1" in r["Kernel_Name"]]
a, b = p1[-6], p1[-5]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r["Kernel_Name"][:80]}')
PY
