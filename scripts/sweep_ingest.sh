#!/bin/bash
# Ingest-kernel variant sweep + PMC traffic passes (one counter group per run).
set -u
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
ARGS="--steps 10 --warmup 3 --no-cpu-baseline"
for agg in sum_i64 count; do
  for u in 1 2 4; do
    GW_INGEST_UNROLL=$u timeout -k 10 300 python -u bench.py $ARGS --agg $agg > gpurun_out/sweep/b_${agg}_u$u.json 2> gpurun_out/sweep/b_${agg}_u$u.err || { echo "bench $agg u$u failed"; tail -5 gpurun_out/sweep/b_${agg}_u$u.err; exit 4; }
    python - "$agg" "$u" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/sweep/b_{sys.argv[1]}_u{sys.argv[2]}.json"))
r=d["roofline"]
print(f"{sys.argv[1]:8s} U={sys.argv[2]} value={d['value']/1e9:6.2f} Gev/s ms/step={d['ms_per_step']:.3f} ingest={r['avg_launch_ms']:.3f}ms frac={r['frac']:.3f} fire={r['fire_avg_launch_ms']:.3f}ms")
PY
  done
done
if [ "${PMC:-1}" = "1" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $ctr | tr ' ' '_')
    timeout -s KILL 180 rocprofv3 --pmc $ctr -d gpurun_out/sweep/pmc_$tag -o run --output-format csv -- python -u bench.py $ARGS > gpurun_out/sweep/pmc_$tag.json 2> gpurun_out/sweep/pmc_$tag.err || { echo "pmc $ctr failed"; tail -5 gpurun_out/sweep/pmc_$tag.err; exit 5; }
  done
  ls -R gpurun_out/sweep | head -30
fi
