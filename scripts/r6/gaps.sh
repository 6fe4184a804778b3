#!/bin/bash
# Idle time inside the headline's timed window: the default bench, then a kernel + HIP API
# trace of the same command and scripts/r6/gaps.py over it.  OUT: gpurun_out/r6/gaps/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/gaps${SUFFIX:-}
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python scripts/r5/jf.py $O/bench.json value ms_per_step roofline.frac roofline.avg_launch_ms
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/trace -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench_trace.json 2> $O/bench_trace.err || { tail -5 $O/bench_trace.err; exit 5; }
python scripts/r6/gaps.py $O/trace/run_kernel_trace.csv $O/bench_trace.json $O/trace/run_hip_api_trace.csv > $O/gaps.txt
cat $O/gaps.txt
python scripts/pipeline_check.py $O/trace/run_kernel_trace.csv $O/bench_trace.json
gzip -f $O/trace/run_hip_api_trace.csv
