#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, wave/LDS counters) over the network-buffer decode
# kernels of scripts/netbuf_bench.py --mode decode; one pass per counter group.
set -u
O=gpurun_out/nbpmc
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "k_nb_" -d $R/$O/pmc_$i -o run --output-format csv -- python -u $R/scripts/netbuf_bench.py --mode decode > $R/$O/p$i.json 2> $R/$O/p$i.err) || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 6; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pmc_*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("<")[0].split("::")[-1]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
