#!/bin/bash
# Decode throughput of the network-buffer ingest, per kernel (rocprofv3 kernel trace):
# the stateless decode at two grid caps and the operator path (scratch reused).
set -u
O=${1:-gpurun_out/nb}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for cfg in "decode 4096" "decode 0" "decode 1024" "operator 4096"; do
  set -- $cfg
  tag=$1_$2
  (cd /tmp && GW_NB_GRID=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$tag -o run --output-format csv -- python -u $R/scripts/netbuf_bench.py --mode $1 > $R/$O/bench_$tag.json 2> $R/$O/bench_$tag.err) || { echo "$tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
  echo "$tag: $(cat $O/bench_$tag.json | cut -c1-200)"
done
