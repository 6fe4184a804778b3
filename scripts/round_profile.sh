#!/bin/bash
# Measurement set of a round (run on the GPU box): default bench with CPU baseline,
# rocprofv3 kernel-trace stats of the same command, PMC traffic passes (one counter
# group per run), LDS counters of the apply kernel.
set -u
R=${ROUND:-r1}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 4; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python -u bench.py > $O/bench_traced.json 2> $O/bench_traced.err || { echo "trace failed"; tail -5 $O/bench_traced.err; exit 5; }
i=0
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "k_rgn|k_fire" -d $O/pmc/pmc_$i -o run --output-format csv -- python -u bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/pmc_$i.json 2> $O/pmc_$i.err || { echo "pmc $ctr failed"; tail -5 $O/pmc_$i.err; exit 6; }
done
python scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
python scripts/traffic.py $O/pmc sum_i64 10000000 $O/traffic.json > /dev/null
echo done
