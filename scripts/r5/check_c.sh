#!/bin/bash
# Packed ingest: parity tests, then the bench's exchange path at N = 1 (--force-exchange) with
# words decoded by pass 1 / unpacked / 24-B records: values and the fired rows' checksum.
set -u
O=gpurun_out/r5/pk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_exchange_pack.py tests/test_gpu_exchange_native.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "Error|error|assert|FAILED" $O/tests.log | head -20; exit $rc; fi
for p in auto unpack off; do
  timeout -k 10 300 python -u bench.py --force-exchange --pack $p --checksum --no-host-fed --no-cpu-baseline > $O/bench_$p.json 2> $O/bench_$p.err || { tail -10 $O/bench_$p.err; exit 4; }
  echo "$p: $(python scripts/r5/jf.py $O/bench_$p.json value ms_per_step rows_checksum exchange_path)"
done
