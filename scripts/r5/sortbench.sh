#!/bin/bash
# Sort microbenchmark over the tile configurations (GW_SORT_CFG) on 25-bit u32 and 40-bit u64 keys.
set -u
mkdir -p gpurun_out/r5/sortb
for c in ${CFGS:-0 2}; do
  for a in "10000000 25 10 0 0" "10000000 25 10 0 1" "10000000 40 5 1 0" "1 25 3 0 1" "4097 9 3 0 1" "100000 17 3 0 0" "10000000 64 3 1 1"; do
    echo "cfg $c [$a]: $(GW_SORT_CFG=$c timeout -k 10 60 scripts/r5/sortbench $a)"
  done
done | tee gpurun_out/r5/sortb/cfgs.txt
