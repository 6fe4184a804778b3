#!/bin/bash
# The N > 1 code path on one GPU (bench.py --force-exchange): bench line, then a kernel + HIP
# API trace of the same command.  OUT: gpurun_out/r6/xtrace${SUFFIX}/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/xtrace${SUFFIX:-}
mkdir -p $O
timeout -k 10 300 python -u bench.py --force-exchange --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python scripts/r5/jf.py $O/bench.json value ms_per_step
timeout -k 10 300 rocprofv3 --kernel-trace ${API_TRACE:-} -d $O/trace -o run --output-format csv -- python3 -u bench.py --force-exchange --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench_trace.json 2> $O/bench_trace.err || { tail -5 $O/bench_trace.err; exit 5; }
[ -f $O/trace/run_hip_api_trace.csv ] && gzip -f $O/trace/run_hip_api_trace.csv
python scripts/r5/jf.py $O/bench_trace.json value ms_per_step
