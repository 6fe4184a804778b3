"""Gaps (us) between the kernels around each fire in a rocprofv3 kernel trace: the flush's
apply -> (status copy | k_fire_guard) -> k_fire2.  usage: fire_gaps.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void ", "").split("<")[0].split("(")[0]
for prev, r in zip(rows, rows[1:]):
    a, b = short(prev["Kernel_Name"]), short(r["Kernel_Name"])
    if "k_fire2" in b or "k_fire_guard" in b or "k_fire_guard" in a:
        gap = (int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3
        print(f"{a:32s} -> {b:24s} {gap:7.1f} us")
