#!/bin/bash
# Region partition placing tiles by atomics for packed batches: exchange tests, fired rows'
# checksum against the stable partition and no exchange, then rate and a kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/unstable
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_native.py tests/test_gpu_exchange_pack.py tests/test_gpu_multirank.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
run() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step rows_checksum)"
}
run ck_unstable GW_PART_STABLE=0 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange --checksum
run ck_stable GW_PART_STABLE=1 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange --checksum
run ck_direct GW_PART_STABLE=0 python -u bench.py --no-host-fed --no-cpu-baseline --checksum
for i in 1 2; do
  run unstable_$i GW_PART_STABLE=0 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange
  run stable_$i GW_PART_STABLE=1 python -u bench.py --no-host-fed --no-cpu-baseline --force-exchange
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py --force-exchange --no-cpu-baseline --no-host-fed > $O/bench_trace.json 2> $O/bench_trace.err || exit 5
grep -E "k_part_regions|k_rgn_p1" $O/trace/run_kernel_stats.csv | cut -c1-160
