#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run; summaries land in gpurun_out/prof_<tag>/
set -u
TAG=${TAG:-r1}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}.err; exit 4; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python -u bench.py ${BENCH_ARGS:-} --no-cpu-baseline > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_${TAG}.err; exit 5; }
find gpurun_out/prof_${TAG} -name "*stats*" | head
for f in $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv"); do head -15 $f; done
