#!/bin/bash
# Round 6 experiment: P2's time when it reads P1 output written just before (a flush per
# batch: GW_BUFFER_RECORDS = one batch) against the bench's 10-batch flush.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/exp1
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
cat $O/bench.json
for v in base flush1; do
  if [ $v = flush1 ]; then export GW_BUFFER_RECORDS=10000000; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 5; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1)
  python scripts/kstats.py $f --top 14 > $O/kstats_$v.txt
  cat $O/kstats_$v.txt
done
