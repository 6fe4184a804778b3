#!/bin/bash
# The exchange finishing 1 or 2 batches ahead of the ingest (bench.py --exchange-ahead) on the
# N > 1 code path at N = 1 (--force-exchange): fired rows' checksum for both and without the
# exchange, then the rate, alternating.  OUT: gpurun_out/r6/ahead/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ahead
mkdir -p $O
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-host-fed --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step rows_checksum)"
}
run ck_a1 --force-exchange --exchange-ahead 1 --checksum
run ck_a2 --force-exchange --exchange-ahead 2 --checksum
run ck_direct --checksum
for i in 1 2; do
  run a1_$i --force-exchange --exchange-ahead 1
  run a2_$i --force-exchange --exchange-ahead 2
done
