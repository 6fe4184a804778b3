#!/bin/bash
# Sort microbenchmark: what each stage costs (GW_SORT_EXP drops stages; results then mismatch).
set -u
mkdir -p gpurun_out/r5/sortb
for c in ${CFGS:-0 2}; do for x in 0 1 2 4 3 7; do
  echo "cfg $c exp $x: $(GW_SORT_CFG=$c GW_SORT_EXP=$x timeout -k 10 60 scripts/r5/sortbench 10000000 25 10 0)"
done; done | tee gpurun_out/r5/sortb/exp.txt
cd /tmp && export TMPDIR=/tmp && GW_SORT_CFG=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5/sortb/prof -o run --output-format csv -- $GRAFT_REPO_ROOT/scripts/r5/sortbench 10000000 25 10 0 > /dev/null
f=$(find $GRAFT_REPO_ROOT/gpurun_out/r5/sortb/prof -name '*kernel_stats.csv' | head -1)
cut -d, -f1-6 $f | head -8
