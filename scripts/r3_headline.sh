#!/bin/bash
# Round-3 headline: the default bench line (as the driver runs it), then a rocprofv3 kernel
# trace of the same workload (no CPU baseline / host-fed legs).  Outputs under gpurun_out/r3/.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TAG=${TAG:-head}
timeout -k 10 400 python3 -u bench.py ${BENCH_ARGS:-} > gpurun_out/r3/${TAG}_bench.json 2> gpurun_out/r3/${TAG}_bench.err || exit $?
head -c 600 gpurun_out/r3/${TAG}_bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/${TAG}_prof -o run --output-format csv -- \
    python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > gpurun_out/r3/${TAG}_prof.json 2> gpurun_out/r3/${TAG}_prof.err || exit $?
python3 scripts/kstats.py gpurun_out/r3/${TAG}_prof/run_kernel_stats.csv --top 12 | grep "gw::" || true
