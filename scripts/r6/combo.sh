#!/bin/bash
# One GPU call: targeted tests, the headline A/B of table loads with kernel traces, E = 10M
# (1M-record batches) for both, the exchange path on one GPU.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/${TAG:-combo}
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 420 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread --durations=12 > $O/tests.log 2>&1
  rc=$?
  tail -22 $O/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
AB=${TAG:-combo} VARIANTS="${VARIANTS}" bash scripts/r6/ab_libs.sh || exit 4
AB=${TAG:-combo}_e10m NO_PROF=1 BENCH_ARGS="--events-per-pane 10000000" VARIANTS="${VARIANTS}" bash scripts/r6/ab_libs.sh || exit 5
TAG=${TAG:-combo}_x NO_PROF=1 bash scripts/r6/xchk.sh || exit 6
