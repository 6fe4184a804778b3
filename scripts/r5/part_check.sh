#!/bin/bash
# Partition kernels (single-pass region partition, tile-ranked scatter, wave-aggregated
# histogram) and the exchange's self-copy: partition / exchange tests, then the exchange path
# on one GPU under a kernel trace, with the region partition (default) and without it.
set -u
O=gpurun_out/r5/part
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_exchange_native.py tests/test_gpu_exchange_pack.py tests/test_gpu_multirank.py \
  tests/test_gpu_discovery.py "tests/test_gpu_parity.py::test_key_groups_and_partition_device" \
  -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
XO=$O/xprof bash scripts/r5/xprof.sh || exit 4
GW_PART_REGIONS=0 XO=$O/xprof_3pass bash scripts/r5/xprof.sh
