#!/bin/bash
# Experiment builds side by side on one box: for each flink_amd/libgpuwin_<tag>.so given
# (tag "base" = the product library), one short bench.py run (no CPU baseline, no
# host-fed leg) -> gpurun_out/exp/<tag>.json.  Stops at the first failure.
set -u
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = base ]; then lib=flink_amd/libgpuwin.so; else lib=flink_amd/libgpuwin_$tag.so; fi
  GW_LIB_PATH=$PWD/$lib timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} \
      > gpurun_out/exp/$tag.json 2> gpurun_out/exp/$tag.err || { echo "$tag failed"; tail -20 gpurun_out/exp/$tag.err; exit 3; }
  python3 scripts/exp_summary.py "$tag" gpurun_out/exp/$tag.json
done
