#!/bin/bash
# rocprofv3 kernel traces of the default bench under env variants (VARIANTS as in r4_ab.sh),
# then (PMC=1) the PMC passes of the first variant.  Output under gpurun_out/r4/prof_<name>/.
set -u
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  name=${v%%=*}; envs=""
  [ "$name" != "$v" ] && envs=${v#*=}
  O=gpurun_out/r4/prof_$name
  mkdir -p $O
  ( [ -n "$envs" ] && export ${envs//,/ }; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
      python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err ) || { echo "$name trace failed"; tail -5 $O/bench.err; exit 5; }
  echo "== $name"; python3 scripts/region_times.py $O/trace/run_kernel_trace.csv
done
[ -n "${PMC:-}" ] || exit 0
v=${VARIANTS%% *}; name=${v%%=*}; envs=""; [ "$name" != "$v" ] && envs=${v#*=}
O=gpurun_out/r4/prof_$name
i=0
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  ( [ -n "$envs" ] && export ${envs//,/ }; timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "k_rgn|k_fire" -d $O/pmc/pmc_$i -o run --output-format csv -- \
      python -u bench.py --no-cpu-baseline --no-host-fed --steps 10 --warmup 2 > $O/pmc_$i.json 2> $O/pmc_$i.err ) || { echo "pmc $ctr failed"; tail -5 $O/pmc_$i.err; exit 6; }
done
python3 scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt 2>&1
cat $O/pmc_summary.txt
