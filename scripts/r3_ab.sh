#!/bin/bash
# A/B of the headline bench between environment settings: for each "TAG=ENV..." in AB
# (space-separated, ENV as VAR=value,VAR=value), a short bench + a rocprofv3 kernel trace.
# Outputs under gpurun_out/r3/ab_<TAG>.*
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
for spec in ${AB:-base=}; do
    tag=${spec%%=*}
    envs=${spec#*=}
    (
        [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
        timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/ab_${tag} -o run --output-format csv -- \
            python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > gpurun_out/r3/ab_${tag}.json 2> gpurun_out/r3/ab_${tag}.err
    ) || { echo "$tag failed"; tail -5 gpurun_out/r3/ab_${tag}.err; exit 5; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/r3/ab_${tag}.json')); r=d['roofline']
print('${tag}', round(d['value']/1e9,2), 'Gev/s frac', round(r['frac'],4), 'p1', round(r['pass1_avg_ms'],4), 'flush', round(r['apply_avg_ms'],4), 'fire', round(r['fire_avg_launch_ms'],4))"
    python3 scripts/kstats.py gpurun_out/r3/ab_${tag}/run_kernel_stats.csv --top 10 2>/dev/null | head -14
done
