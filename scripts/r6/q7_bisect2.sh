#!/bin/bash
# Q7 (tumbling max) with the trees of round 5's end (ee7e025) and 85f3321 against the current one.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6/q7bisect2
mkdir -p $O
for v in r5 85f cur; do
  d=$PWD; [ $v != cur ] && d=$PWD/_old/$v
  ( cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$v -o run --output-format csv -- python -u scripts/configs_bench.py --only q7 --no-cpu-baseline --steps 30 > $O/q7_$v.jsonl 2> $O/q7_$v.err ) || { echo "$v failed"; grep -v rocprof $O/q7_$v.err | tail -3; continue; }
  f=$(find $O/t_$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(python scripts/r5/jf.py $O/q7_$v.jsonl value) $(grep -E 'apply_nar|k_rgn_p2|k_fire2' $f | awk -F, '{print $1, $3, $4}' | tr '\n' ' ')"
done
