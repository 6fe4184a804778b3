"""Cross-check bench.py's HIP-event pipeline time against rocprofv3's kernel trace of the
same command: device time of the ingest-pipeline kernels (k_rgn_p1 per batch; plan / P2 /
apply per flush) divided by the k_rgn_p1 dispatches in the timed window, taken as the
dispatches after the warmup flush (the 'apply' dispatches bracket the timed region)."""
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
b = json.loads(open(bench).read().strip().splitlines()[-1])
rows = [r for r in csv.DictReader(open(trace)) if "gw::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void gw::", "").replace("gw::", "").split("<")[0]
APPLY = ("k_rgn_apply", "k_rgn_apply_nar")
applies = [i for i, r in enumerate(rows) if name(r) in APPLY]
# bench: warmup, flush (apply #k), timed steps (fires flush), final flush (last apply)
steps, warm = b["steps"], b["warmup"]
p1_idx = [i for i, r in enumerate(rows) if name(r) == "k_rgn_p1"]
first_timed_p1 = p1_idx[warm]
start = max(i for i in applies if i < first_timed_p1)
last_timed_p1 = p1_idx[warm + steps - 1]
# the fire's flush after the last timed batch, and bench's closing gw_flush right behind it (the
# ring positions the last fire left carried): every apply before the next pass 1 (a host-fed
# leg may follow)
nxt = min([i for i in p1_idx if i > last_timed_p1] + [len(rows)])
end = max(i for i in applies if last_timed_p1 < i < nxt)
dur = {}
for r in rows[start + 1:end + 1]:
    n = name(r)
    dur.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
pipe = ["k_rgn_p1", "k_rgn_plan1", "k_rgn_plan2", "k_rgn_plan3", "k_rgn_p2", "k_rgn_apply", "k_rgn_apply_nar"]
tot = sum(sum(dur.get(k, [])) for k in pipe)
nb = len(dur.get("k_rgn_p1", []))
print(f"timed batches (k_rgn_p1 dispatches): {nb} (bench steps {steps})")
for k in pipe + ["k_fire", "k_fire2"]:
    v = dur.get(k, [])
    if v:
        print(f"  {k:14s} dispatches {len(v):3d}  avg {sum(v) / len(v):8.4f} ms  total {sum(v):8.3f} ms")
print(f"rocprof pipeline ms per batch: {tot / max(nb, 1):.4f}")
print(f"bench.py HIP-event pipeline ms per batch (roofline.avg_launch_ms): {b['roofline']['avg_launch_ms']:.4f}")
