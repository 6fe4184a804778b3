#!/bin/bash
# Targeted GPU tests (TESTS), then the A/B of library builds (scripts/r6/ab_libs.sh).
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/${TAG:-step}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread --durations=15 > $O/tests.log 2>&1
  rc=$?
  tail -25 $O/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
[ -n "${VARIANTS:-}" ] && AB=${TAG:-step} bash scripts/r6/ab_libs.sh
exit 0
