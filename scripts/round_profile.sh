#!/bin/bash
# Full measurement set for one round: default bench (with CPU baseline), rocprofv3
# kernel-trace stats of the same command, PMC traffic passes, microbenchmarks.
set -u
R=${ROUND:-r1}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 4; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python -u bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || { echo "trace failed"; exit 5; }
for ctr in FETCH_SIZE WRITE_SIZE "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d $O/pmc_$tag -o run --output-format csv -- python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/pmc_$tag.json 2> $O/pmc_$tag.err || { echo "pmc $ctr failed"; tail -5 $O/pmc_$tag.err; exit 6; }
done
timeout -k 10 120 ./flink_amd/_build/ingest_probe > $O/ingest_probe.txt 2>&1 || exit 7
timeout -k 10 120 ./flink_amd/_build/mall_probe > $O/mall_probe.txt 2>&1 || exit 8
echo done
