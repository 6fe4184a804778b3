#!/bin/bash
# gpurun with bounded retries ONLY when no box/slot was available (nothing ran, nothing charged)
LOG=$1; shift
for i in 1 2 3 4 5 6; do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && grep -qE "no free box|slot\(s\) on this pod are busy" $LOG; then
    sleep 150; continue
  fi
  exit $rc
done
exit $rc
