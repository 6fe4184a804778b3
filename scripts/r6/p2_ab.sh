#!/bin/bash
# P2 prefetch A/B: region-path parity subset, then the headline bench alternating the new
# library with flink_amd/libgpuwin_base.so (the previous tree), with a kernel trace of each.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ab_${AB:-p2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_headline.py tests/test_gpu_region_compact.py} -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
AB=${AB:-p2} VARIANTS="new=default base=flink_amd/libgpuwin_base.so" bash scripts/r6/ab_libs.sh || exit $?
AB=${AB:-p2}_2 NO_PROF=1 VARIANTS="new=default base=flink_amd/libgpuwin_base.so" bash scripts/r6/ab_libs.sh
