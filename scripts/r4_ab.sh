#!/bin/bash
# A/B of bench.py (default headline, no CPU baseline / host-fed legs) over environment variants:
# VARIANTS="name=ENV=val,ENV2=val2 name2=..." ("base" = no extra env).  Each variant runs
# RUNS times (default 2).  Results under gpurun_out/r4/ab_<name>_<i>.json.
set -u
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  name=${v%%=*}; envs=""
  [ "$name" != "$v" ] && envs=${v#*=}
  for i in $(seq 1 ${RUNS:-2}); do
    ( [ -n "$envs" ] && export ${envs//,/ }; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} \
        > gpurun_out/r4/ab_${name}_$i.json 2> gpurun_out/r4/ab_${name}_$i.err ) || { echo "$name run $i failed"; tail -20 gpurun_out/r4/ab_${name}_$i.err; exit 4; }
    python3 - gpurun_out/r4/ab_${name}_$i.json $name <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(f"{sys.argv[2]:>10} value {d['value']/1e9:.2f} G/s ms/step {d['ms_per_step']:.4f} frac {r['frac']:.4f} "
              f"p1 {r['pass1_avg_ms']:.4f} flush {r['apply_avg_ms']:.4f} x{r['apply_launches']} fire {r['fire_avg_launch_ms']:.4f}")
PY
  done
done
