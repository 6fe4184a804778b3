#!/bin/bash
# The one-GPU exchange path with the exchange on its own stream vs on the operator's stream.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/xstream
mkdir -p $O
for st in own operator; do
  timeout -k 10 300 python -u bench.py --force-exchange --pack auto --no-host-fed --no-cpu-baseline --exchange-stream $st > $O/bench_$st.json 2> $O/bench_$st.err || { tail -10 $O/bench_$st.err; exit 4; }
  echo "$st: $(python scripts/r5/jf.py $O/bench_$st.json value ms_per_step)"
done
timeout -k 10 300 python -u bench.py --force-exchange --pack auto --no-host-fed --no-cpu-baseline --exchange-stream operator --checksum > $O/bench_operator_ck.json 2> $O/bench_operator_ck.err || exit 5
echo "operator checksum: $(python scripts/r5/jf.py $O/bench_operator_ck.json rows_checksum)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/xprof -o run --output-format csv -- python -u bench.py --force-exchange --pack auto --no-host-fed --no-cpu-baseline --exchange-stream operator > $O/xprof.json 2> $O/xprof.err || exit 6
python scripts/kstats.py $(find $O/xprof -name "*kernel_stats.csv" | head -1) --top 12
