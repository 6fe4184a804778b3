#!/bin/bash
# Sort microbenchmark (default shapes), pre-aggregation + session + first-element parity,
# then the ysb and sessions configs.
set -u
mkdir -p gpurun_out/r5/a
export TMPDIR=/tmp
for a in "10000000 26 10 0 1" "10000000 40 5 1 1" "10000000 64 3 1 1" "4097 9 3 0 1" "100000 17 3 0 0"; do
  echo "sort [$a]: $(timeout -k 10 60 scripts/r5/sortbench $a)"
done | tee gpurun_out/r5/a/sort.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lateness.py tests/test_gpu_session_scenarios.py tests/test_gpu_session_snapshot.py tests/test_gpu_count_windows.py tests/test_gpu_first_element.py tests/test_gpu_minmaxby.py ${EXTRA:-} -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/a/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5/a/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/a/tests.log | head -20; exit $rc; fi
timeout -k 10 400 python -u scripts/configs_bench.py --only ${ONLY:-ysb,sessions,q7_first} --steps 30 --no-cpu-baseline > gpurun_out/r5/a/configs.jsonl 2> gpurun_out/r5/a/configs.err || { tail -20 gpurun_out/r5/a/configs.err; exit 4; }
python - <<'PY'
import json
for ln in open("gpurun_out/r5/a/configs.jsonl"):
    if ln.startswith("{"):
        d = json.loads(ln); r = d.get("roofline") or {}
        print(d["config"], d.get("value"), d.get("ms_per_step"), r.get("frac"), r.get("launch_ms"))
PY
