#!/bin/bash
# 8192-record P1 tiles / P2 rounds (experiment builds) against the default 4096: the headline
# parity test on each build, then bench + kernel trace per build.  OUT: gpurun_out/r6/ab_tile/
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ab_tile
mkdir -p $O
for v in t8k1024 t8k512; do
  GW_LIB_PATH=$PWD/flink_amd/libgpuwin_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -q -x --timeout 240 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 $O/tests_$v.log)"
  [ $rc -ne 0 ] && exit $rc
done
AB=tile VARIANTS="base=default t8k1024=flink_amd/libgpuwin_t8k1024.so t8k512=flink_amd/libgpuwin_t8k512.so" bash scripts/r6/ab_libs.sh
