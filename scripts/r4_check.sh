#!/bin/bash
# Round-4 GPU check: the given GPU tests (TESTS), then bench.py (BENCH_ARGS) unless NOBENCH is
# set.  Logs under gpurun_out/r4/.
set -u
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
TAG=${TAG:-chk}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout ${PER_TEST:-300} --timeout-method thread \
      --durations=0 -m gpu ${K:+-k "$K"} $TESTS > gpurun_out/r4/pytest_${TAG}.log 2>&1
  rc=$?
  tail -25 gpurun_out/r4/pytest_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/r4/bench_${TAG}.json 2> gpurun_out/r4/bench_${TAG}.err
rc=$?
python3 - gpurun_out/r4/bench_${TAG}.json <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line); r = d["roofline"]
        print(f"value {d['value']/1e9:.2f} G/s ms/step {d['ms_per_step']:.4f} frac {r['frac']:.4f} p1 {r['pass1_avg_ms']:.4f} "
              f"flush {r['apply_avg_ms']:.4f} x{r['apply_launches']} fire {r['fire_avg_launch_ms']:.4f}")
        for k in ("rows_checksum", "oracle_check", "host_fed", "cpu_baseline"):
            if k in d: print(k, d[k])
PY
exit $rc
