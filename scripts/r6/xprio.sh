#!/bin/bash
# The exchange's own stream at high HIP priority against the default (--force-exchange).
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/xprio
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step)"
}
for i in 1 2; do
  run p0_$i
  run phigh_$i --exchange-priority -1
done
