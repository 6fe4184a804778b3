"""One line per experiment bench JSON: throughput and the pipeline's per-kernel times."""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(f"{tag:>12}: {d['value'] / 1e9:6.2f} G ev/s  {d['ms_per_step']:.3f} ms/step  frac={r.get('frac', 0):.3f} "
      f"p1={r.get('pass1_avg_ms', 0):.4f} flush={r.get('apply_avg_ms', 0):.3f}/{r.get('apply_launches')} "
      f"fire={r.get('fire_avg_launch_ms', 0):.3f}/{r.get('fire_launches')}")
