#!/bin/bash
# Region partition variants: its GPU test, then the one-GPU exchange path under a kernel trace.
set -u
O=gpurun_out/r5/part2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_exchange_pack.py -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
XO=$O/xprof bash scripts/r5/xprof.sh
