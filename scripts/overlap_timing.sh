#!/bin/bash
# Timing of the overlapped vs serial exchange in the two-rank gloo rehearsal (one GPU), alternated.
set -u
mkdir -p gpurun_out/overlap
export TMPDIR=/tmp
ARGS="--gpus 2 --dist-backend gloo --keys 1000000 --events-per-pane 10000000 --steps 40 --warmup 5 --no-cpu-baseline"
i=0
for ov in on off on off; do
  i=$((i+1))
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29520 + i)) bench.py $ARGS --overlap $ov > gpurun_out/overlap/t_${i}_$ov.json 2> gpurun_out/overlap/t_${i}_$ov.err \
    || { echo "overlap=$ov failed"; tail -30 gpurun_out/overlap/t_${i}_$ov.err; exit 4; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/overlap/t_${i}_$ov.json').read().strip().splitlines()[-1]); print('$ov', round(d['ms_per_step'],3))"
done
