#!/bin/bash
# PMC passes over the default bench for the nar1 kernels (one counter group per pass).
set -u
O=gpurun_out/r5/pmc_n1
mkdir -p $O
export TMPDIR=/tmp
KRE=${KRE:-k_rgn_apply_n1|k_rgn_p1n}
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$KRE" -d $O/pmc_$i -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed --steps 10 > $O/p$i.json 2> $O/p$i.err || { echo "pmc pass $i ($ctr) failed"; tail -5 $O/p$i.err; exit 6; }
done
python scripts/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
