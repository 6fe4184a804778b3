#!/bin/bash
# fastfire.sh, then the exchange-stream A/B (xstream.sh) in the same call.
set -u
bash scripts/r6/fastfire.sh || exit $?
GW_HOST_PROFILE=1 bash scripts/r6/xstream.sh
