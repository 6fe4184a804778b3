#!/bin/bash
# Round 6 measurement set (GPU box): the headline's rocprofv3 kernel trace + PMC passes at the
# bench's own cadence (scripts/headline_profile.sh) -> traffic.json, installed as
# profiles/r6/traffic.json for the bench line; then the default bench (CPU baseline and
# host-fed legs included) and the cross-check of its HIP-event pipeline time against the trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/${FINAL:-final}
mkdir -p $O profiles/r6
TAG=r6/${FINAL:-final} bash scripts/headline_profile.sh > $O/headline_profile.log 2>&1 || { tail -20 $O/headline_profile.log; exit 4; }
tail -12 $O/headline_profile.log
cp $O/traffic.json profiles/r6/traffic.json
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 5; }
cat $O/bench.json
python scripts/pipeline_check.py $O/trace/run_kernel_trace.csv $O/bench_trace.json > $O/pipeline_check.txt; cat $O/pipeline_check.txt
if [ -n "${E10M:-}" ]; then
  timeout -k 10 300 python -u bench.py --events-per-pane 10000000 --warmup 15 --no-cpu-baseline --no-host-fed > $O/bench_e10m.json 2> $O/bench_e10m.err || { tail -20 $O/bench_e10m.err; exit 6; }
  python scripts/r5/jf.py $O/bench_e10m.json value ms_per_step roofline.frac
fi
