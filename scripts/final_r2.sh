#!/bin/bash
# Round-2 measurement set on one MI355X box: full GPU test suite, smoke, the default bench
# (CPU baseline + host-fed leg), its rocprofv3 kernel trace, PMC traffic passes at the
# bench's cadence, and the other BASELINE configs with their CPU baselines.
set -u
O=gpurun_out/final
if [ -n "${ONLY_CONFIGS:-}" ]; then
  mkdir -p $O
  timeout -k 10 900 python -u scripts/configs_bench.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 6; }
  cat $O/configs.jsonl
  exit 0
fi
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
cat $O/bench.json
TAG=final/hl bash scripts/headline_profile.sh > $O/headline_profile.log 2>&1 || { tail -20 $O/headline_profile.log; exit 5; }
tail -30 $O/headline_profile.log
[ -n "${SKIP_CONFIGS:-}" ] && exit 0
timeout -k 10 900 python -u scripts/configs_bench.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 6; }
cat $O/configs.jsonl
