"""Print fields of the last JSON line of a file: python scripts/r5/jf.py FILE FIELD[.SUB] ..."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
out = []
for f in sys.argv[2:]:
    v = d
    for k in f.split("."):
        v = v.get(k) if isinstance(v, dict) else None
    out.append(f"{f}={v}")
print(" ".join(out))
