#!/bin/bash
# PMC traffic of the headline pipeline at the bench's own cadence (default steps: 25 batches,
# flushes every 10): FETCH_SIZE and WRITE_SIZE in separate passes, then traffic.py.
set -u
O=gpurun_out/${ROUND:-r5/final}
mkdir -p $O/pmcfull
export TMPDIR=/tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-include-regex "k_rgn|k_fire" -d $O/pmcfull/pmc_$i -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed > $O/pmcfull_$i.json 2> $O/pmcfull_$i.err || { echo "pmc $ctr failed"; tail -5 $O/pmcfull_$i.err; exit 6; }
done
python scripts/traffic.py $O/pmcfull sum_i64 10000000 $O/traffic_full.json
python scripts/pmc_summary.py $O/pmcfull > $O/pmcfull_summary.txt 2>&1
