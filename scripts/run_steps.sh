#!/bin/bash
# Run GPU steps in order under their own time limits; stop at the first step that crashes,
# aborts, faults or times out (exit codes other than 0 and 1), per the pool's rules.
# Usage: scripts/run_steps.sh "<seconds>|<name>|<command>" ...
# Each step's output goes to gpurun_out/<name>.log.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
