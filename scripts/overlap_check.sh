#!/bin/bash
# Two-rank rehearsal of the exchanged bench on one GPU (gloo moves the columns through the
# host): the overlapped (double-buffered) and the serial exchange must fire the same rows.
set -u
mkdir -p gpurun_out/overlap
export TMPDIR=/tmp
ARGS="--gpus 2 --dist-backend gloo --keys 1000000 --events-per-pane 10000000 --steps 20 --warmup 5 --checksum --no-cpu-baseline"
for ov in off on; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py $ARGS --overlap $ov > gpurun_out/overlap/bench_$ov.json 2> gpurun_out/overlap/bench_$ov.err \
    || { echo "overlap=$ov failed"; tail -30 gpurun_out/overlap/bench_$ov.err; exit 4; }
  cat gpurun_out/overlap/bench_$ov.json
done
python - <<'EOF'
import json
r = {ov: json.loads(open(f"gpurun_out/overlap/bench_{ov}.json").read().strip().splitlines()[-1]) for ov in ("off", "on")}
print("rows_fired", {k: (v["rows_fired"], v["rows_checksum"]) for k, v in r.items()}, "value", {k: round(v["value"] / 1e9, 3) for k, v in r.items()})
assert (r["off"]["rows_fired"], r["off"]["rows_checksum"]) == (r["on"]["rows_fired"], r["on"]["rows_checksum"]), "overlap changed the fired rows"
EOF
