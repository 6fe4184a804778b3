#!/bin/bash
# Headline (bench.py default) profile: rocprofv3 kernel stats, then PMC passes (one
# counter group per pass) over the region pipeline and the fire sweep; outputs under
# gpurun_out/$TAG.
set -u
TAG=${TAG:-hl}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-fed > $O/bench_trace.json 2> $O/bench_trace.err || { echo "trace failed"; tail -5 $O/bench_trace.err; exit 5; }
python3 scripts/kstats.py $O/trace/run_kernel_stats.csv --top 16
KRE="k_rgn|k_fire" TAG=$TAG/pmc PMC_PGRPS="${PMC_PGRPS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS}" bash scripts/pmc_kernel.sh || exit 6
python3 scripts/traffic.py $O/pmc sum_i64 10000000 $O/traffic.json && cat $O/traffic.json
