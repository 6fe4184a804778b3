#!/bin/bash
# Packed exchange on the GPU: device partition / unpack, native exchange, world size 2; then
# the ysb pre-aggregation stage-drop A/B.
set -u
mkdir -p gpurun_out/r5/x
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_pack.py tests/test_gpu_exchange_native.py tests/test_gpu_multirank.py tests/test_gpu_nar_carry.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r5/x/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5/x/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" gpurun_out/r5/x/tests.log | head -20; exit $rc; fi
SKIP_SORTB=1 ONLY=ysb VARS="${VARS:-default GW_PREAGG_EXP=1 GW_PREAGG_EXP=2 GW_PREAGG_EXP=3}" bash scripts/r5/sess_ab.sh
