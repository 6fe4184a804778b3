#!/bin/bash
# The headline bench with round 5's final tree (ee7e025) against the current one, alternating.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6/hlr5
mkdir -p $O
for i in 1 2 3; do
  for v in r5 cur; do
    d=$PWD; [ $v != cur ] && d=$PWD/_old/$v
    ( cd $d && timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-fed > $O/hl_${v}_$i.json 2> $O/hl_${v}_$i.err ) || { echo "$v failed"; tail -3 $O/hl_${v}_$i.err; exit 4; }
    echo "$v $i $(python scripts/r5/jf.py $O/hl_${v}_$i.json value roofline.pass1_avg_ms roofline.apply_avg_ms roofline.fire_avg_launch_ms)"
  done
done
