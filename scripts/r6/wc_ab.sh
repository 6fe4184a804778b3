#!/bin/bash
# Count-window table sizing A/B: count-window parity suite, then the WindowWordCount config
# line with the new library and flink_amd/libgpuwin_base.so, alternating.  OUT: gpurun_out/r6/wc/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/wc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_count_windows.py -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
for tag in new base new2 base2; do
  case $tag in base*) export GW_LIB_PATH=$PWD/flink_amd/libgpuwin_base.so;; *) unset GW_LIB_PATH;; esac
  timeout -k 10 300 python -u scripts/configs_bench.py --only wordcount ${CB_ARGS:-} > $O/wc_$tag.jsonl 2> $O/wc_$tag.err || { tail -20 $O/wc_$tag.err; exit 4; }
  python -c "import json;d=json.loads(open('$O/wc_$tag.jsonl').read().strip().splitlines()[-1]);print('$tag',round(d['value']/1e9,3),'G',round(d['ms_per_step'],4),'ms')"
done
unset GW_LIB_PATH
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u scripts/configs_bench.py --only wordcount > $O/wc_prof.jsonl 2> $O/wc_prof.err || { tail -5 $O/wc_prof.err; exit 5; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_wordcount.csv
