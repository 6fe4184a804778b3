#!/bin/bash
# Region buffer limit: Q7 (50-batch tumbling windows) and the headline at 2^27 (default) and
# 2^29 records (GW_BUFFER_RECORDS), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/buflimit
mkdir -p $O
for i in 1 2; do
  for L in 134217728 536870912; do
    GW_BUFFER_RECORDS=$L timeout -k 10 400 python -u scripts/configs_bench.py --only q7 --no-cpu-baseline > $O/q7_${L}_$i.jsonl 2> $O/q7_${L}_$i.err || { tail -5 $O/q7_${L}_$i.err; exit 4; }
    GW_BUFFER_RECORDS=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > $O/hl_${L}_$i.json 2> $O/hl_${L}_$i.err || { tail -5 $O/hl_${L}_$i.err; exit 5; }
    echo "L=$L $i q7 $(python scripts/r5/jf.py $O/q7_${L}_$i.jsonl value) hl $(python scripts/r5/jf.py $O/hl_${L}_$i.json value)"
  done
done
