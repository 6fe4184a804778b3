#!/bin/bash
# Session region-path experiments: for each GW_SP_EXP value in EXPS, a short sessions bench
# under a rocprofv3 kernel trace.  Outputs under gpurun_out/r3/spexp_<v>*.
set -u
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
for v in ${EXPS:-0 1 2}; do
    GW_SESSION_PATH=region GW_SP_EXP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3/spexp_$v -o run --output-format csv -- \
        python3 -u scripts/configs_bench.py --only sessions --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
        > gpurun_out/r3/spexp_$v.log 2> gpurun_out/r3/spexp_$v.err || { echo "exp $v failed"; tail -3 gpurun_out/r3/spexp_$v.err; exit 3; }
    echo "== exp $v"; grep "sp_keys exp" gpurun_out/r3/spexp_$v.err | tail -2
    python3 scripts/kstats.py gpurun_out/r3/spexp_$v/run_kernel_stats.csv --top 12 | grep "gw::"
done
