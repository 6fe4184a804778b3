#!/bin/bash
# The exchange driven from a host thread of its own (bench.py --exchange-driver thread) against
# the inline driver, on the N > 1 code path at N = 1 (--force-exchange): fired rows' checksum
# for both and without the exchange, then the rate, alternating.  OUT: gpurun_out/r6/feeder/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/feeder
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_native.py tests/test_gpu_exchange_pack.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
run() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --no-host-fed --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -10 $O/bench_$n.err; exit 4; }
  echo "$n: $(python scripts/r5/jf.py $O/bench_$n.json value ms_per_step rows_checksum)"
}
run ck_thread --force-exchange --checksum
run ck_inline --force-exchange --exchange-driver inline --checksum
run ck_direct --checksum
for i in 1 2; do
  run thread_$i --force-exchange
  run inline_$i --force-exchange --exchange-driver inline
done
