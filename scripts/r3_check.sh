#!/bin/bash
# Round-3 GPU check: the given GPU tests (TESTS, default: the key-type / reference-snapshot /
# exchange set), then the bench.  Logs under gpurun_out/r3/.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_gpu_refsnap.py tests/test_gpu_snapshot.py tests/test_jni_glue.py tests/test_gpu_exchange_native.py tests/test_gpu_multirank.py"}
TAG=${TAG:-keys}
timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/r3/pytest_${TAG}.log 2>&1
rc=$?
tail -5 gpurun_out/r3/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/r3/bench_${TAG}.json 2> gpurun_out/r3/bench_${TAG}.err
rc=$?
head -c 700 gpurun_out/r3/bench_${TAG}.json
exit $rc
