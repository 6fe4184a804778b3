#!/bin/bash
# gpurun with bounded retries ONLY on gpurun's transient status (no box / slot, a box lost while being
# prepared: nothing of the command ran, nothing charged)
LOG=$1; shift
for i in 1 2 3 4 5 6; do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then
    sleep 150; continue
  fi
  exit $rc
done
exit $rc
