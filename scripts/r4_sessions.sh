#!/bin/bash
# Sessions config: configs_bench.py --only sessions under a rocprofv3 kernel trace, per session
# ingest path (PATHS, default "region sort").  Output under gpurun_out/r4/sess_<path>/.
set -u
export TMPDIR=/tmp
for p in ${PATHS:-region sort}; do
  O=gpurun_out/r4/sess_$p
  mkdir -p $O
  GW_SESSION_PATH=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
      python3 -u scripts/configs_bench.py --only sessions ${CB_ARGS:-} > $O/bench.log 2> $O/bench.err
  rc=$?
  tail -2 $O/bench.log
  [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
  python3 scripts/kstats.py $O/trace/run_kernel_stats.csv 2>/dev/null | head -14 || true
done
