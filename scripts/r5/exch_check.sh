#!/bin/bash
# Exchange-side GPU tests after a partition change, then smoke().
set -u
O=gpurun_out/r5/exch_check
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_exchange_native.py tests/test_gpu_exchange_pack.py tests/test_gpu_multirank.py \
  tests/test_gpu_discovery.py "tests/test_gpu_parity.py::test_key_groups_and_partition_device" \
  -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -1 $O/smoke.log
