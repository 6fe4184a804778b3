#!/bin/bash
# Sessions config: the sort path against the region path (short runs under a rocprofv3 kernel
# trace, GW_SP_EXP=3 prints the region path's slow-slot reasons).  gpurun_out/r3/sab_<path>*.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
for p in ${PATHS:-sort region}; do
    GW_SESSION_PATH=$p GW_SP_EXP=${SP_EXP:-3} timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/sab_$p -o run --output-format csv -- \
        python3 -u scripts/configs_bench.py --only sessions --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline \
        > gpurun_out/r3/sab_$p.log 2> gpurun_out/r3/sab_$p.err || { echo "$p failed"; tail -3 gpurun_out/r3/sab_$p.err; exit 3; }
    echo "== $p"; grep -o '"value": [0-9.e+]*' gpurun_out/r3/sab_$p.log; grep "sp_keys" gpurun_out/r3/sab_$p.err | tail -1
    python3 scripts/kstats.py gpurun_out/r3/sab_$p/run_kernel_stats.csv --top 14 | grep "gw::\|rocprim"
done
