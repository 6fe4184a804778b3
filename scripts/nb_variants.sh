#!/bin/bash
# Network-buffer decode kernels per experiment library (flink_amd/libgpuwin_<tag>.so, "base" =
# the product library; "name@VAR=v,VAR2=w" = the product library with those environment
# settings): rocprofv3 kernel stats of scripts/netbuf_bench.py --mode decode.
set -u
O=gpurun_out/nbv
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for tag in "$@"; do
  envs=""
  case "$tag" in
    *@*) envs=${tag#*@}; tag=${tag%%@*}; lib=$R/flink_amd/libgpuwin.so ;;
    base) lib=$R/flink_amd/libgpuwin.so ;;
    *) lib=$R/flink_amd/libgpuwin_$tag.so ;;
  esac
  (cd /tmp && { [ -z "$envs" ] || export ${envs//,/ }; } && GW_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/$tag -o run --output-format csv -- python -u $R/scripts/netbuf_bench.py --mode decode > $R/$O/$tag.json 2> $R/$O/$tag.err) || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 - "$O/$tag" "$tag" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
print(sys.argv[2], " ".join(f"{r['Name'].split('<')[0].split('::')[-1]}={float(r['AverageNs'])/1000:.1f}" for r in csv.DictReader(open(f)) if "nb_" in r["Name"]))
PY
done
