#!/bin/bash
# nar1 (single-pass narrow flush) + k_fire2 check: parity suites over the narrow two-pass
# path and the fire, then the headline bench: default, GW_NAR1=0 (P2 path), GW_FIRE2=0.
set -u
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_region_narrow.py tests/test_gpu_headline.py tests/test_gpu_parity.py ${EXTRA_TESTS:-} -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/nar1_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5/nar1_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/nar1_tests.log | head -20; exit $rc; fi
for v in default GW_NAR1=0 GW_FIRE2=0; do
  tag=${v//=/_}
  env $([ $v = default ] || echo $v) timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench_$tag.json 2> gpurun_out/r5/bench_$tag.err || { tail -20 gpurun_out/r5/bench_$tag.err; exit 4; }
  echo "$tag: $(python scripts/r5/jf.py gpurun_out/r5/bench_$tag.json value ms_per_step roofline.frac roofline.avg_launch_ms roofline.pass1_avg_ms roofline.apply_avg_ms)"
done
