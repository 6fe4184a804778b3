#!/bin/bash
# Hand-written sort: session / count-window / first-element / lateness parity, then the
# sessions config (configs_bench) for the speed.
set -u
bash scripts/r5/sortbench.sh || exit 9
mkdir -p gpurun_out/r5/sess
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_session_snapshot.py tests/test_gpu_session_scenarios.py tests/test_gpu_session_deferred.py tests/test_gpu_session_groups.py tests/test_gpu_count_windows.py tests/test_gpu_first_element.py tests/test_gpu_minmaxby.py tests/test_gpu_lateness.py tests/test_gpu_parity.py -k "${K:-}" -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/sess/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5/sess/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/sess/tests.log | head -20; exit $rc; fi
timeout -k 10 400 python -u scripts/configs_bench.py --only ${ONLY:-sessions,q7_first,q7_maxby} > gpurun_out/r5/sess/configs.jsonl 2> gpurun_out/r5/sess/configs.err || { tail -20 gpurun_out/r5/sess/configs.err; exit 4; }
python - <<'PY'
import json
for ln in open("gpurun_out/r5/sess/configs.jsonl"):
    if ln.startswith("{"):
        d = json.loads(ln); print(d.get("config", {}).get("workload", d.get("name")), d.get("value"), d.get("ms_per_step"), (d.get("roofline") or {}).get("frac"))
PY
