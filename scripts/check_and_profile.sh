#!/bin/bash
# Parity tests (stop on crash) then a kernel-trace profile of the default bench.
set -u
TAG=${TAG:-dev}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python -u bench.py ${BENCH_ARGS:-} --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_${TAG}.err; exit 5; }
cat gpurun_out/bench_prof_${TAG}.json
for f in $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -20; done
