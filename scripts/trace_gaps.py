"""Idle gaps on the device between consecutive kernels (rocprofv3 kernel trace CSV):
prints the last N kernels with their duration and the idle time before each, then the
total busy / idle time over that window."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
last = max(i for i, r in enumerate(rows) if "gw::" in r["Kernel_Name"])
rows = rows[: last + 1][-n:]
busy = idle = 0
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1000 if prev_end is not None else 0.0
    if prev_end is not None:
        idle += max(0, s - prev_end)
    busy += e - s
    prev_end = max(prev_end or 0, e)
    print(f"gap {gap:8.1f}  dur {(e - s) / 1000:8.1f} us  {r['Kernel_Name'][:60]}")
print(f"window: busy {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us")
