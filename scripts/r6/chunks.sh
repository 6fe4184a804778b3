#!/bin/bash
# Two-stream flush (P2 of bucket chunk c+1 beside the apply of chunk c): parity at the bench's
# cadence and the region-path suites, then the bench at GW_FLUSH_CHUNKS = 1 / 2 / 4 / 8 and a
# kernel trace of the default.  OUT: gpurun_out/r6/chunks/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/chunks
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_nar_carry.py tests/test_gpu_fast_fire.py tests/test_gpu_region_narrow.py tests/test_gpu_region_compact.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for K in ${KS:-1 4 2 8}; do
  GW_FLUSH_CHUNKS=$K timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > $O/bench_k$K.json 2> $O/bench_k$K.err || { tail -20 $O/bench_k$K.err; exit 4; }
  echo "K=$K $(python scripts/r5/jf.py $O/bench_k$K.json value ms_per_step roofline.frac roofline.apply_avg_ms)"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-fed > $O/bench_trace.json 2> $O/bench_trace.err || { tail -5 $O/bench_trace.err; exit 5; }
python scripts/r6/gaps.py $O/trace/run_kernel_trace.csv $O/bench_trace.json > $O/gaps.txt
head -30 $O/gaps.txt
