#!/bin/bash
# Round-5 closing check: the packing / partition tests and the one-GPU exchange profile, the
# whole GPU suite + smoke, then the default bench line.
set -u
bash scripts/r5/part_ab.sh || exit 3
ROUND=r5/suite4 bash scripts/r5/gpu_suite.sh || exit 4
O=gpurun_out/r5/final4
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 5; }
python scripts/r5/jf.py $O/bench.json value ms_per_step
