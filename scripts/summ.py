"""One-line summary of bench.py JSON output files (ingest pipeline split)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    r = d["roofline"]
    print(f"{f}: {d['value'] / 1e9:.2f} Gev/s frac {r['frac']:.4f} p1 {r['pass1_avg_ms']:.4f} "
          f"apply {r['apply_avg_ms']:.4f} x{r['apply_launches']} fire {r['fire_avg_launch_ms']:.4f} "
          f"ms/step {d['ms_per_step']:.4f}")
