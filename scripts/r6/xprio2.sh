#!/bin/bash
# The operator's stream at the greatest HIP priority (experiment build) on the N > 1 path and the
# headline, against the default build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/xprio2
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-host-fed --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step)"
}
for i in 1 2; do
  unset GW_LIB_PATH; run x_def_$i --force-exchange
  export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_xhi.so; run x_hi_$i --force-exchange
done
unset GW_LIB_PATH; run hl_def
export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_xhi.so; run hl_hi
