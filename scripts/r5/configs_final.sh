#!/bin/bash
# Every BASELINE config line (configs_bench.py, CPU baselines included), then each config's
# kernel-trace stats under rocprofv3 (the same command without the CPU baseline), so each line's
# frac can be recomputed from the kernel times beside it.
set -u
O=gpurun_out/${ROUND:-r5/configs}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u scripts/configs_bench.py --only ${ONLY:-wordcount,ysb,q7,q7_first,q7_maxby,sessions} > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 4; }
python scripts/r5/jf.py $O/configs.jsonl value
for c in ${ONLY:-wordcount ysb q7 q7_first q7_maxby sessions}; do
  c=${c//,/ }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$c -o run --output-format csv -- python -u scripts/configs_bench.py --only $c --no-cpu-baseline > $O/traced_$c.jsonl 2> $O/traced_$c.err || { tail -5 $O/traced_$c.err; exit 5; }
  echo "traced $c"
done
