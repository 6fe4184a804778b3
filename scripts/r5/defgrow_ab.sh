#!/bin/bash
# Deferred-list growth A/B (GW_DEF_GROW=0: the round-4 policy) at E = 10M and at the headline,
# with the host-time profile.
set -u
O=gpurun_out/r5/defgrow
mkdir -p $O
for v in ${VARS:-default GW_DEF_GROW=0}; do
  tag=${v//=/_}
  for e in 10000000 100000000; do
    env GW_HOST_PROFILE=1 $([ $v = default ] || echo $v) timeout -k 10 300 python -u bench.py --events-per-pane $e --no-host-fed --no-cpu-baseline > $O/${tag}_$e.json 2> $O/${tag}_$e.err || { tail -5 $O/${tag}_$e.err; exit 3; }
    echo "$tag E=$e: $(python scripts/r5/jf.py $O/${tag}_$e.json value ms_per_step) $(grep -E 'deferred|status-wait' $O/${tag}_$e.err | tr -s ' ' | tr '\n' ' ')"
  done
done
