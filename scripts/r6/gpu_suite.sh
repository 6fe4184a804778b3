#!/bin/bash
# Full GPU suite with per-test durations, then the default bench (one line) and a kernel trace
# of the bench for the pipeline cross-check.  OUT: gpurun_out/r6/<tag>/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/${TAG:-suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread --durations=80 ${PYTEST_ARGS:-} > $O/gpu_suite.log 2>&1
rc=$?
tail -5 $O/gpu_suite.log
[ $rc -ne 0 ] && exit $rc
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
cat $O/bench.json
