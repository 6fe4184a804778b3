#!/bin/bash
# Parity subset (TESTS), then alternating A/B of the default library against
# flink_amd/libgpuwin_base.so at the headline and at E = 10M events per pane.
set -u
export TMPDIR=/tmp
O=gpurun_out/r6/ab_${AB:-x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS} -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
NO_PROF=1 VARIANTS="new=default base=flink_amd/libgpuwin_base.so new2=default base2=flink_amd/libgpuwin_base.so" bash scripts/r6/ab_libs.sh
AB=${AB:-x}_e10m BENCH_ARGS="--events-per-pane 10000000 --warmup 15" NO_PROF=1 VARIANTS="new=default base=flink_amd/libgpuwin_base.so new2=default base2=flink_amd/libgpuwin_base.so" bash scripts/r6/ab_libs.sh
