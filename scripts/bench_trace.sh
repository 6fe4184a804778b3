#!/bin/bash
# bench.py (default headline) + a rocprofv3 kernel trace of the same command; per-kernel
# durations of the region pipeline.  TAG names the output directory under gpurun_out/.
set -u
TAG=${TAG:-bt}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 4
python3 - gpurun_out/$TAG/bench.json <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(f"value {d['value']/1e9:.2f} G/s ms/step {d['ms_per_step']:.4f} frac {r['frac']:.4f} p1 {r['pass1_avg_ms']:.4f} flush {r['apply_avg_ms']:.4f} fire {r['fire_avg_launch_ms']:.4f}")
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/trace -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-host-fed ${BENCH_ARGS:-} > gpurun_out/$TAG/bench_trace.json 2> gpurun_out/$TAG/bench_trace.err || exit 5
python3 scripts/region_times.py gpurun_out/$TAG/trace/run_kernel_trace.csv
