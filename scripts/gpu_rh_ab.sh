#!/bin/bash
# A/B of the sort-free rolling COUNT ablations (scripts/rolling_hist_ab.py), one process each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-rh_ab}; mkdir -p "$out"; shift
export PYTHONPATH=$PWD
for cfg in "$@"; do  # cfg = ABLATE[:KEYS[:FILT[:SORT_FREE]]]
  IFS=: read -r a k f sf <<< "$cfg"
  MXS_RH_ABLATE=$a KEYS=${k:-10000} FILT=${f:-1} SORT_FREE=${sf:-1} timeout -k 10 120 python scripts/rolling_hist_ab.py >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit $?
done
cat "$out/ab.jsonl"
