"""Device timeline of bench.py's timed region from a rocprofv3 kernel trace: from the
first k_rgn_p1 after the warmup flush to the last gw:: kernel; busy time per kernel
name and the idle gaps between kernels."""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
gw = [i for i, r in enumerate(rows) if "gw::" in r["Kernel_Name"]]
last = gw[-1]
p1 = [i for i in gw if "k_rgn_p1" in rows[i]["Kernel_Name"]]
first = p1[-steps]
win = rows[first:last + 1]
busy = collections.Counter()
calls = collections.Counter()
idle = 0
prev_end = None
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    busy[name] += e - s
    calls[name] += 1
    if prev_end is not None and s > prev_end:
        idle += s - prev_end
    prev_end = max(prev_end or 0, e)
span = int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])
print(f"span {span / 1e3:.1f} us  idle {idle / 1e3:.1f} us  per step {span / 1e3 / steps:.1f} us")
for k, v in busy.most_common():
    print(f"{k:42s} {calls[k]:4d} calls {v / 1e3:9.1f} us")
