"""Where the device is idle inside bench.py's timed window: every gap between consecutive
kernels of a rocprofv3 kernel trace (all kernels, copies included), summed by the (previous,
next) kernel pair, plus the host's blocking HIP calls over the same window when an API trace
is given.  The timed window is bracketed as in pipeline_check.py (the flush before the first
timed k_rgn_p1, the flush after the last).
usage: gaps.py kernel_trace.csv bench.json [hip_api_trace.csv]"""
import collections
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
b = json.loads(open(bench).read().strip().splitlines()[-1])
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("void ", "").replace("gw::", "").split("<")[0].split("(")[0][:28]
p1 = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_rgn_p1"]
applies = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]).startswith("k_rgn_apply")]
steps, warm = b["steps"], b["warmup"]
start = max(i for i in applies if i < p1[warm])
end = min(i for i in applies if i > p1[warm + steps - 1])
win = rows[start:end + 1]
t0, t1 = int(win[0]["End_Timestamp"]), int(win[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win[1:])
gaps = collections.defaultdict(lambda: [0, 0.0, 0.0])
for prev, r in zip(win, win[1:]):
    g = (int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3
    k = (short(prev["Kernel_Name"]), short(r["Kernel_Name"]))
    gaps[k][0] += 1
    gaps[k][1] += max(g, 0.0)
    gaps[k][2] = max(gaps[k][2], g)
span = (t1 - t0) / 1e3
print(f"window: {steps} steps, {span:.1f} us span, kernels busy {busy / 1e3:.1f} us, idle {span - busy / 1e3:.1f} us "
      f"({(span - busy / 1e3) / steps:.2f} us per step)")
print(f"{'previous':28s} -> {'next':28s} {'n':>4s} {'sum us':>9s} {'max us':>8s}")
for k, (n, s, mx) in sorted(gaps.items(), key=lambda kv: -kv[1][1]):
    print(f"{k[0]:28s} -> {k[1]:28s} {n:4d} {s:9.1f} {mx:8.1f}")
if len(sys.argv) > 3:
    api = [r for r in csv.DictReader(open(sys.argv[3]))
           if t0 <= int(r["Start_Timestamp"]) <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in api:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[r["Function"]][0] += 1
        agg[r["Function"]][1] += d
    print(f"\nHIP API calls inside the window ({len(api)}):")
    for f, (n, s) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"  {f:36s} {n:5d} {s:9.1f} us")
    # the host's calls during every long idle stretch: what the device was waiting for
    print("\nHIP API calls during idle gaps > 20 us (offsets from the previous kernel's end):")
    for prev, r in zip(win, win[1:]):
        e, s = int(prev["End_Timestamp"]), int(r["Start_Timestamp"])
        if (s - e) / 1e3 <= 20:
            continue
        print(f"  gap {short(prev['Kernel_Name'])} -> {short(r['Kernel_Name'])}: {(s - e) / 1e3:.1f} us")
        for c in api:
            cs, ce = int(c["Start_Timestamp"]), int(c["End_Timestamp"])
            if ce >= e - 5000 and cs <= s:
                print(f"      {(cs - e) / 1e3:8.1f} .. {(ce - e) / 1e3:8.1f}  {c['Function']}")
