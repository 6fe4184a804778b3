"""Per-dispatch durations of the region pipeline and the fire sweep from a rocprofv3
kernel trace (run_kernel_trace.csv): median P1, and per-flush P2 / apply, fire."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for name in ("k_rgn_p1", "k_publish_status", "k_rgn_p2", "k_rgn_apply", "k_fire", "k_merge_deferred"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    if d:
        print(f"{name:18s} n={len(d):3d} median={statistics.median(d):8.1f} us  all={[round(x) for x in d[:14]]}")
