#!/bin/bash
# PMC passes over the sessions config (region ingest), kernels matching $KRE; one counter
# group per pass.  Summary under gpurun_out/$TAG/summary.txt.
set -u
KRE=${KRE:-k_sp_}
TAG=${TAG:-sesspmc}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
i=0
IFS=';' read -ra PGRPS <<< "${PMC_PGRPS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR;TCC_HIT_sum TCC_MISS_sum}"
for ctr in "${PGRPS[@]}"; do
  i=$((i+1))
  GW_SESSION_PATH=region timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$KRE" -d $O/pmc_$i -o run --output-format csv -- python3 -u scripts/configs_bench.py --only sessions --steps 6 --warmup 2 --no-cpu-baseline > $O/p$i.log 2> $O/p$i.err || { echo "pmc pass $i ($ctr) failed"; tail -5 $O/p$i.err; exit 6; }
done
python3 scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
