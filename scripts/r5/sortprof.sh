#!/bin/bash
# Per-kernel times of one sort configuration (rocprofv3 kernel trace of the microbenchmark).
set -u
mkdir -p gpurun_out/r5/sortb
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in ${CFGS:-0 2}; do
  GW_SORT_CFG=$c timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/sortb/prof$c -o run --output-format csv -- $R/scripts/r5/sortbench 10000000 25 10 0 ${IOTA:-1} || exit 3
  f=$(find $R/gpurun_out/r5/sortb/prof$c -name '*kernel_stats.csv' | head -1)
  echo "cfg $c"; cut -d, -f1-4 $f | head -8
done
