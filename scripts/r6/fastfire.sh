#!/bin/bash
# The fire enqueued behind its flush: its tests, the headline test, then the A/B against a
# GW_FAST_FIRE=0 build (bench line + kernel trace each).  OUT: gpurun_out/r6/fastfire/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/fastfire
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast_fire.py tests/test_gpu_headline.py tests/test_gpu_nar_carry.py -q -x --timeout 300 --timeout-method thread --durations=10 > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
[ $rc -ne 0 ] && exit $rc
AB=fastfire VARIANTS="on=default off=flink_amd/libgpuwin_noff.so" bash scripts/r6/ab_libs.sh
