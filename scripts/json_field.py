"""Print one field of the last JSON line of a file: python scripts/json_field.py FILE FIELD[.SUB]"""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
for k in sys.argv[2].split("."):
    d = d[k]
print(json.dumps(d))
