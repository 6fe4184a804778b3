#!/bin/bash
# Sessions config A/B over environment variants (VARS), then session parity (K selects tests).
set -u
mkdir -p gpurun_out/r5/sab
export TMPDIR=/tmp
[ -n "${SKIP_SORTB:-}" ] || CFGS="0 2" bash scripts/r5/sortbench.sh
for v in ${VARS:-default}; do
  tag=${v//=/_}; tag=${tag//,/_}
  env $(echo $v | tr ',' ' ' | sed 's/default//') timeout -k 10 300 python -u scripts/configs_bench.py --only ${ONLY:-sessions} --steps 40 --no-cpu-baseline > gpurun_out/r5/sab/$tag.jsonl 2> gpurun_out/r5/sab/$tag.err || { tail -20 gpurun_out/r5/sab/$tag.err; exit 4; }
  echo "$tag: $(python scripts/r5/jf.py gpurun_out/r5/sab/$tag.jsonl value ms_per_step roofline.launch_ms.ingest)"
done
[ -n "${TESTS:-}" ] || exit 0
timeout -k 10 800 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/sab/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5/sab/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/sab/tests.log | head -20; exit $rc; fi
