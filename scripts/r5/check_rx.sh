#!/bin/bash
# Fired rows' checksum of the bench stream through the exchange path with the region partition
# (packed words decoded by pass 1 / unpacked / 24-B records), the three-pass partition, and
# without the exchange: all must agree.
set -u
O=gpurun_out/r5/rx
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, env, args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step rows_checksum exchange_path)"
}
for p in auto unpack off; do
  run regions_$p GW_PART_REGIONS=1 python -u bench.py --force-exchange --pack $p --checksum --no-host-fed --no-cpu-baseline
done
run threepass_auto GW_PART_REGIONS=0 python -u bench.py --force-exchange --pack auto --checksum --no-host-fed --no-cpu-baseline
run direct GW_PART_REGIONS=1 python -u bench.py --checksum --no-host-fed --no-cpu-baseline
