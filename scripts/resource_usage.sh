#!/bin/bash
# Per-kernel register / scratch / LDS / occupancy of every HIP source, from the compiler's
# kernel-resource-usage remarks, one line per kernel -> profiles/${ROUND:-r3}/resource_usage/<src>.txt
set -eu
cd "$(dirname "$0")/.."
out=profiles/${ROUND:-r3}/resource_usage
mkdir -p "$out"
for src in flink_amd/csrc/*.hip; do
    b=$(basename "$src" .hip)
    /opt/rocm/bin/hipcc -O3 -std=c++17 -munsafe-fp-atomics --offload-arch=gfx950 -x hip -c "$src" -o /tmp/ru_$b.o \
        -Rpass-analysis=kernel-resource-usage 2>&1 |
        awk '/Function Name:/ {if (line) print line; sub(/.*remark: /, ""); sub(/ \[-Rpass.*/, ""); line=$0; next}
             /VGPRs: |ScratchSize|Occupancy|LDS Size/ {sub(/.*remark: +/, ""); sub(/ \[-Rpass.*/, ""); line=line "\t" $0}
             END {if (line) print line}' > "$out/$b.txt"
    echo "$b: $(wc -l < "$out/$b.txt") kernels, $(awk -F'ScratchSize \\[bytes/lane\\]: ' '{split($2,a,"\t"); if (a[1]+0>0) n++} END {print n+0}' "$out/$b.txt") with scratch"
done
