#!/usr/bin/env bash
# AMD GPU discovery for Flink's external-resource framework.
#
# Drop-in for flink-external-resources/flink-external-resource-gpu's
# nvidia-gpu-discovery.sh (src/main/resources/nvidia-gpu-discovery.sh:21-55): same
# arguments, same output, so GPUDriver (GPUDriverOptions.DISCOVERY_SCRIPT_PATH /
# DISCOVERY_SCRIPT_ARG) runs it unchanged:
#
#   amd-gpu-discovery.sh gpu-amount [--enable-coordination-mode] [--coordination-file path]
#
# prints the indices of `gpu-amount` MI355X devices as "0,1,..." on stdout and exits 0,
# or prints "Could not get enough GPU resources." and exits 1.  Indices are HIP device
# ordinals (the order HIP_VISIBLE_DEVICES / gw_config.device use).  Devices come from
# `amd-smi list --csv`, else `rocm-smi --showid --csv`, else the KFD topology (GPU nodes
# are those with simd_count > 0).
#
# Coordination mode (several TaskManagers on one host): a lock-protected file holds
# "index pid" lines; an index whose owner process is gone is taken over.
set -u

usage() {
  echo "Usage: ./amd-gpu-discovery.sh gpu-amount [--enable-coordination-mode] [--coordination-file filePath]"
}

[ $# -lt 1 ] && { usage; exit 1; }
AMOUNT=$1
shift
COORDINATE=0
COORD_FILE=/var/tmp/flink-gpu-coordination
while [ $# -ge 1 ]; do
  case "$1" in
    --enable-coordination-mode) COORDINATE=1 ;;
    --coordination-file) shift; COORD_FILE=${1:-$COORD_FILE} ;;
    *) ;;  # unknown options are ignored, as the NVIDIA script does
  esac
  shift
done
case "$AMOUNT" in ''|*[!0-9]*) usage; exit 1 ;; esac
[ "$AMOUNT" -eq 0 ] && exit 0

list_devices() {
  local out
  # amd-smi: header "gpu,gpu_bdf,gpu_uuid,..." then one row per device
  if out=$(amd-smi list --csv 2>/dev/null) && [ -n "$out" ]; then
    echo "$out" | awk -F, 'NR > 1 && $1 ~ /^[0-9]+$/ { print $1 }'
    return 0
  fi
  # rocm-smi: rows "card0,..." after a "device,..." header
  if out=$(rocm-smi --showid --csv 2>/dev/null) && [ -n "$out" ]; then
    echo "$out" | awk -F, 'NR > 1 && $1 ~ /^card[0-9]+$/ { sub("card", "", $1); print $1 }'
    return 0
  fi
  # KFD topology: GPU nodes in node order are the HIP ordinals
  local d i=0
  for d in /sys/class/kfd/kfd/topology/nodes/*; do
    [ -r "$d/properties" ] || continue
    if awk '$1 == "simd_count" && $2 > 0 { f = 1 } END { exit !f }' "$d/properties"; then
      echo $i
      i=$((i + 1))
    fi
  done
}

mapfile -t DEVICES < <(list_devices | sort -n | uniq)

fail() { echo "Could not get enough GPU resources."; exit 1; }
join() { local IFS=,; echo "$*"; }

if [ "$COORDINATE" -eq 0 ]; then
  [ "${#DEVICES[@]}" -lt "$AMOUNT" ] && fail
  join "${DEVICES[@]:0:$AMOUNT}"
  exit 0
fi

touch "$COORD_FILE" 2>/dev/null || fail
OWNER=$PPID  # the TaskManager process that runs the script
(
  flock -x 9
  picked=()
  # 1) free indices, 2) indices whose recorded owner has exited
  for pass in free stale; do
    for dev in "${DEVICES[@]}"; do
      [ "${#picked[@]}" -eq "$AMOUNT" ] && break 2
      owner=$(awk -v d="$dev" '$1 == d { print $2; exit }' "$COORD_FILE")
      if [ "$pass" = free ] && [ -z "$owner" ]; then
        picked+=("$dev")
      elif [ "$pass" = stale ] && [ -n "$owner" ] && ! kill -0 "$owner" 2>/dev/null; then
        awk -v d="$dev" '$1 != d' "$COORD_FILE" > "$COORD_FILE.tmp.$$" && cat "$COORD_FILE.tmp.$$" > "$COORD_FILE"
        rm -f "$COORD_FILE.tmp.$$"
        picked+=("$dev")
      fi
    done
  done
  [ "${#picked[@]}" -lt "$AMOUNT" ] && fail
  for dev in "${picked[@]}"; do echo "$dev $OWNER" >> "$COORD_FILE"; done
  join "${picked[@]}"
) 9<"$COORD_FILE"
