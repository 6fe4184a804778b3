#!/bin/bash
# rocprofv3 kernel-trace stats of one short bench run (no CPU baseline); summary to
# gpurun_out/prof_${TAG}/.
set -u
TAG=${TAG:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_prof_${TAG}.json 2> gpurun_out/bench_prof_${TAG}.err || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_${TAG}.err; exit 5; }
cat gpurun_out/bench_prof_${TAG}.json
for f in $(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -24; done
