#!/bin/bash
# Session-window experiment builds side by side: configs_bench sessions (12.5M keys, avg_f64)
# per flink_amd/libgpuwin_<tag>.so ("base" = the product library) -> gpurun_out/exp/sess_<tag>.json
set -u
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = base ]; then lib=flink_amd/libgpuwin.so; else lib=flink_amd/libgpuwin_$tag.so; fi
  GW_LIB_PATH=$PWD/$lib timeout -k 10 240 python3 -u scripts/configs_bench.py --only sessions --no-cpu-baseline \
      --steps ${SESS_STEPS:-40} > gpurun_out/exp/sess_$tag.json 2> gpurun_out/exp/sess_$tag.err \
      || { echo "$tag failed"; tail -20 gpurun_out/exp/sess_$tag.err; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(f'{sys.argv[1]:>8}: {d[\"value\"]/1e9:6.2f} G ev/s {d[\"ms_per_step\"]:.3f} ms/step')" $tag gpurun_out/exp/sess_$tag.json
done
