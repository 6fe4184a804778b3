#!/bin/bash
# Sessions config timing breakdown of the bucketed path: GW_SB_EXP=2 (P3 gathers only), 1
# (+ sort and heads), 0 (full replay), each a short configs_bench run with kernel timing (the
# rows of the variants are invalid by design); then (PMC=1) one PMC pass over k_sb_replay.
set -u
export TMPDIR=/tmp
O=gpurun_out/r4/sess_exp
mkdir -p $O
for e in ${EXPS:-2 1 0}; do
  GW_SB_EXP=$e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/exp$e -o run --output-format csv -- \
      python3 -u scripts/configs_bench.py --only sessions --steps ${STEPS:-30} --no-cpu-baseline > $O/exp$e.log 2> $O/exp$e.err
  rc=$?
  [ $rc -eq 0 ] || { echo "exp $e failed rc=$rc"; tail -5 $O/exp$e.err; exit $rc; }
  echo "== exp $e"; python3 scripts/kstats.py $O/exp$e/run_kernel_stats.csv --top 6 | grep -E "k_sb|k_sess|kernel "
done
[ -n "${PMC:-}" ] || exit 0
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU \
    --kernel-include-regex "k_sb" -d $O/pmc_1 -o run --output-format csv -- \
    python3 -u scripts/configs_bench.py --only sessions --steps 10 --no-cpu-baseline > $O/pmc.log 2> $O/pmc.err
rc=$?
[ $rc -eq 0 ] || { echo "pmc failed rc=$rc"; tail -5 $O/pmc.err; exit $rc; }
python3 scripts/pmc_summary.py $O > $O/pmc_summary.txt 2>&1; cat $O/pmc_summary.txt
