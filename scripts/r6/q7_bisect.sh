#!/bin/bash
# Q7 (tumbling max) across library builds: the config line and the apply's kernel time.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/q7bisect
mkdir -p $O
for v in r5 85f 019 cur; do
  if [ $v = cur ]; then unset GW_LIB_PATH; else export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$v -o run --output-format csv -- python -u scripts/configs_bench.py --only q7 --no-cpu-baseline --steps 30 > $O/q7_$v.jsonl 2> $O/q7_$v.err || { echo "$v failed"; tail -5 $O/q7_$v.err; continue; }
  f=$(find $O/t_$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(python scripts/r5/jf.py $O/q7_$v.jsonl value) $(grep -E 'apply_nar|k_rgn_p2|k_fire2' $f | awk -F, '{print $1, $3, $4}' | tr '\n' ' ')"
done
