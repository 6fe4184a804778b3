#!/bin/bash
# The exchange on the operator's stream (serialised with its kernels) finishing 1 or 2 batches
# ahead, against its own stream.  OUT: gpurun_out/r6/xstream2/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/xstream2
mkdir -p $O
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step)"
}
for i in 1 2; do
  run own1_$i
  run op1_$i --exchange-stream operator
  run op2_$i --exchange-stream operator --exchange-ahead 2
done
