#!/bin/bash
# A/B of library builds on the default bench: VARIANTS="tag:path ..." (path empty = default library).
set -u
mkdir -p gpurun_out/r5/ab
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/ab/tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r5/ab/tests.log
  if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/ab/tests.log | head -20; exit $rc; fi
fi
for rep in ${REPS:-1 2}; do
for v in $VARIANTS; do
  tag=${v%%:*}; lib=${v#*:}
  env ${lib:+GW_LIB_PATH=$lib} ${ENVS:-} timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > gpurun_out/r5/ab/$tag.$rep.json 2> gpurun_out/r5/ab/$tag.$rep.err || { tail -20 gpurun_out/r5/ab/$tag.$rep.err; exit 4; }
  echo "$tag#$rep: $(python scripts/r5/jf.py gpurun_out/r5/ab/$tag.$rep.json value roofline.frac roofline.avg_launch_ms roofline.pass1_avg_ms roofline.apply_avg_ms)"
done
done
