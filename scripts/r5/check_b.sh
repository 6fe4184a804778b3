#!/bin/bash
# First-element join (range-limited sorts) and session prep (4 records per thread): parity,
# then configs A/B, then Q5 at E = 10M events per pane.
set -u
mkdir -p gpurun_out/r5/b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_first_element.py tests/test_gpu_minmaxby.py tests/test_gpu_session_scenarios.py tests/test_gpu_count_windows.py tests/test_gpu_session_snapshot.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5/b/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/b/tests.log | head -20; exit $rc; fi
for v in default GW_PREP_U=1; do
  tag=${v//=/_}
  env $([ $v = default ] || echo $v) timeout -k 10 400 python -u scripts/configs_bench.py --only sessions,wordcount,q7_first --steps 30 --no-cpu-baseline > gpurun_out/r5/b/cfg_$tag.jsonl 2> gpurun_out/r5/b/cfg_$tag.err || { tail -20 gpurun_out/r5/b/cfg_$tag.err; exit 4; }
  python - gpurun_out/r5/b/cfg_$tag.jsonl $tag <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln); print(sys.argv[2], d["config"], round(d["value"] / 1e9, 2), "G", round(d["ms_per_step"], 3), "ms", (d.get("roofline") or {}).get("launch_ms"))
PY
done
timeout -k 10 300 python -u bench.py --events-per-pane 10000000 --no-host-fed --cpu-baseline-seconds 5 > gpurun_out/r5/b/bench_e10m.json 2> gpurun_out/r5/b/bench_e10m.err || { tail -10 gpurun_out/r5/b/bench_e10m.err; exit 5; }
python scripts/r5/jf.py gpurun_out/r5/b/bench_e10m.json value ms_per_step roofline.frac roofline.fire_avg_launch_ms
