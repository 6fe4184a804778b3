#!/bin/bash
# PMC passes over the default bench restricted to kernels matching $KRE; one pass per
# counter group (gfx950 slot limits), each under its own kill timer.
set -u
KRE=${KRE:-k_rgn_apply}
TAG=${TAG:-pmc}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
i=0
IFS=';' read -ra PGRPS <<< "${PMC_PGRPS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS}"
for ctr in "${PGRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$KRE" -d $O/pmc_$i -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed ${PMC_BENCH_ARGS:-} > $O/p$i.json 2> $O/p$i.err || { echo "pmc pass $i ($ctr) failed"; tail -5 $O/p$i.err; exit 6; }
done
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
