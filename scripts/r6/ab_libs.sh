#!/bin/bash
# A/B of library builds on the headline bench: for each "tag=libpath", the bench line and a
# rocprofv3 kernel trace of the same command, then the timed-window kernel times
# (scripts/pipeline_check.py).  OUT: gpurun_out/r6/ab_<AB>/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ab_${AB:-x}
mkdir -p $O
for spec in $VARIANTS; do
  tag=${spec%%=*}; lib=${spec#*=}
  if [ "$lib" != default ]; then export GW_LIB_PATH=$PWD/$lib; else unset GW_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; exit 4; }
  python -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$tag',round(d['value']/1e9,2),'G',round(d['ms_per_step'],4),'ms frac',round(r['frac'],4),'p1',round(r['pass1_avg_ms'],4),'apply',round(r['apply_avg_ms'],4),'fire',round(r['fire_avg_launch_ms'],4))"
  if [ -z "${NO_PROF:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- python -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > $O/benchprof_$tag.json 2> $O/benchprof_$tag.err || { tail -20 $O/benchprof_$tag.err; exit 5; }
    f=$(find $O/prof_$tag -name "*kernel_trace.csv" | head -1)
    python scripts/pipeline_check.py $f $O/benchprof_$tag.json > $O/pipeline_$tag.txt && cat $O/pipeline_$tag.txt
  fi
done
