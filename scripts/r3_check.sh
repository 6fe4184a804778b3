#!/bin/bash
# Round-3 GPU check: the staging probe, the key-type / reference-snapshot tests, the bench.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
timeout -k 10 180 ./flink_amd/csrc/tools/stage_probe > gpurun_out/r3/stage_probe.txt 2>&1 || { echo "probe failed"; exit 3; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_refsnap.py tests/test_gpu_snapshot.py tests/test_jni_glue.py ${EXTRA_TESTS:-} > gpurun_out/r3/pytest_keys.log 2>&1
rc=$?
tail -5 gpurun_out/r3/pytest_keys.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r3/bench_base.json 2> gpurun_out/r3/bench_base.err
rc=$?
cat gpurun_out/r3/bench_base.json | head -c 600
exit $rc
