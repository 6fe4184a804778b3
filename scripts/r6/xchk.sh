#!/bin/bash
# The N > 1 exchange path on one GPU (bench.py --force-exchange: a one-rank RCCL communicator,
# every record partitioned, exchanged and ingested through the hand-off stream, now one batch
# ahead through gw_exchange_begin / gw_exchange_finish): rate and the fired rows' checksum,
# which must equal the direct path's.  Then a kernel trace of the exchange path.
set -u
O=gpurun_out/r6/${TAG:-xchk}
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step rows_checksum)"
}
run x_auto --force-exchange --pack auto --checksum --no-host-fed --no-cpu-baseline
run direct --checksum --no-host-fed --no-cpu-baseline
run x_rate --force-exchange --pack auto --no-host-fed --no-cpu-baseline
if [ -z "${NO_PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/xprof -o run --output-format csv -- python -u bench.py --force-exchange --pack auto --no-host-fed --no-cpu-baseline > $O/xprof.json 2> $O/xprof.err || { tail -10 $O/xprof.err; exit 5; }
  python scripts/kstats.py $(find $O/xprof -name "*kernel_stats.csv" | head -1) --top 16
fi
