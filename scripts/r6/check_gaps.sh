#!/bin/bash
# Quick parity (bench-cadence headline, fast fire, carry, region suites) then the gap analysis.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/gaps${SUFFIX:-}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_headline.py tests/test_gpu_nar_carry.py tests/test_gpu_fast_fire.py} -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r6/gaps.sh
