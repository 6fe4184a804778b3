#!/bin/bash
# The BASELINE configs besides the headline, each under a rocprofv3 kernel trace: the
# configs_bench.py line (with roofline) per config, and bench.py at E = 10M events per pane
# (1M-event batches: SURVEY §8d's other sweep point).  Output: gpurun_out/r4/configs/<name>/
# (bench line + kernel stats); the lines are collected into gpurun_out/r4/configs/configs.jsonl.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4/configs
mkdir -p $O
: > $O/configs.jsonl
for c in ${CONFIGS:-q7 ysb sessions wordcount q7_first q7_maxby}; do
  mkdir -p $O/$c
  timeout -k 10 ${CFG_TIMEOUT:-240} rocprofv3 --kernel-trace --stats -d $O/$c/trace -o run --output-format csv -- \
      python3 -u scripts/configs_bench.py --only $c ${CB_ARGS:-} > $O/$c/bench.log 2> $O/$c/bench.err
  rc=$?
  [ $rc -eq 0 ] || { echo "$c failed rc=$rc"; tail -5 $O/$c/bench.err; exit $rc; }
  grep '^{' $O/$c/bench.log | tail -1 >> $O/configs.jsonl
  python3 scripts/kstats.py $O/$c/trace/run_kernel_stats.csv --top 12 > $O/$c/kernel_stats.txt 2>&1 || true
  echo "== $c"; tail -c 600 $O/$c/bench.log; head -8 $O/$c/kernel_stats.txt
done
if [ -z "${NO_E10M:-}" ]; then
  mkdir -p $O/q5_e10m
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/q5_e10m/trace -o run --output-format csv -- \
      python3 -u bench.py --events-per-pane 10000000 --steps 100 --warmup 20 --no-host-fed > $O/q5_e10m/bench.json 2> $O/q5_e10m/bench.err
  rc=$?
  [ $rc -eq 0 ] || { echo "q5_e10m failed rc=$rc"; tail -5 $O/q5_e10m/bench.err; exit $rc; }
  grep '^{' $O/q5_e10m/bench.json | tail -1 >> $O/configs.jsonl
  python3 scripts/kstats.py $O/q5_e10m/trace/run_kernel_stats.csv --top 12 > $O/q5_e10m/kernel_stats.txt 2>&1 || true
  echo "== q5_e10m"; head -8 $O/q5_e10m/kernel_stats.txt
fi
