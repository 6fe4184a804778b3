#!/bin/bash
# Sessions config A/B over library builds (GW_LIB_PATH): VARIANTS="name=/path/lib.so ..." ("base": in-tree lib).
set -u
mkdir -p gpurun_out/r4
for v in ${VARIANTS:-base}; do
  name=${v%%=*}; lib=""
  [ "$name" != "$v" ] && lib=${v#*=}
  ( [ -n "$lib" ] && export GW_LIB_PATH=$lib; timeout -k 10 240 python3 -u scripts/configs_bench.py --only sessions --no-cpu-baseline \
      > gpurun_out/r4/sab_$name.log 2> gpurun_out/r4/sab_$name.err ) || { echo "$name failed"; tail -5 gpurun_out/r4/sab_$name.err; exit 4; }
  echo "$name $(python3 scripts/json_field.py gpurun_out/r4/sab_$name.log value) $(python3 scripts/json_field.py gpurun_out/r4/sab_$name.log roofline.device_ms_per_step)"
done
