"""Summarise rocprofv3 --pmc CSVs per kernel (median per dispatch) -> text."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
out = []
for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not name.startswith("void gw::"):
            continue
        short = name.split("(")[0].replace("void gw::", "")
        vals[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(vals.items()):
        out.append(f"{k:32s} {c:24s} dispatches={len(v):3d} median={statistics.median(v):16.1f}")
print("\n".join(out))
