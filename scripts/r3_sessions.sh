#!/bin/bash
# Round-3 session-path check: the session GPU tests, then the sessions config bench (and a
# rocprofv3 kernel trace of it).  Logs under gpurun_out/r3/.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TAG=${TAG:-sess}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    -k "${K:-session or sess}" ${TESTS:-tests/test_gpu_session_region.py tests/test_gpu_parity.py tests/test_gpu_lateness.py tests/test_gpu_snapshot.py tests/test_gpu_restore.py tests/test_gpu_session_groups.py} \
    > gpurun_out/r3/pytest_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/r3/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
GW_SESSION_PATH=${SP_PATH:-region} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/${TAG}_prof -o run --output-format csv -- \
    python3 -u scripts/configs_bench.py --only sessions ${CB_ARGS:-} > gpurun_out/r3/${TAG}_bench.log 2> gpurun_out/r3/${TAG}_bench.err
rc=$?
tail -3 gpurun_out/r3/${TAG}_bench.log
exit $rc
