#!/bin/bash
# Sessions config (sort path) through experiment builds side by side: for each tag,
# flink_amd/libgpuwin_<tag>.so ("base" = the product library) -> gpurun_out/exp/sess_<tag>.json.
set -u
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = base ]; then lib=flink_amd/libgpuwin.so; else lib=flink_amd/libgpuwin_$tag.so; fi
  GW_LIB_PATH=$PWD/$lib timeout -k 10 240 python3 -u scripts/configs_bench.py --only sessions --steps ${STEPS:-60} \
      --warmup 3 --no-cpu-baseline > gpurun_out/exp/sess_$tag.json 2> gpurun_out/exp/sess_$tag.err \
      || { echo "$tag failed"; tail -5 gpurun_out/exp/sess_$tag.err; exit 3; }
  echo "$tag $(grep -o '"value": [0-9.e+]*' gpurun_out/exp/sess_$tag.json)"
done
