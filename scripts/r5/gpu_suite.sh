#!/bin/bash
# The whole GPU suite (one process), then smoke(); progress goes to gpurun_out as it runs.
set -u
O=gpurun_out/${ROUND:-r5/suite}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 500 --timeout-method thread ${EXTRA:-} > $O/suite.log 2>&1
rc=$?
tail -5 $O/suite.log
grep -E "^FAILED|^ERROR" $O/suite.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -2 $O/smoke.log
