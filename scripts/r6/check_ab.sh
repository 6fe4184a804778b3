#!/bin/bash
# Parity subset (TESTS), then an alternating A/B of the default library against
# flink_amd/libgpuwin_base.so (the previous commit's build).  OUT: gpurun_out/r6/ab_$AB/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ab_${AB:-x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_headline.py tests/test_gpu_fast_fire.py} -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
NO_PROF=1 VARIANTS="new=default base=flink_amd/libgpuwin_base.so new2=default base2=flink_amd/libgpuwin_base.so new3=default base3=flink_amd/libgpuwin_base.so" bash scripts/r6/ab_libs.sh
