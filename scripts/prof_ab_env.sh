#!/bin/bash
# Kernel-time A/B of an environment switch over bench.py: prof_ab_env.sh VAR=VALUE_A VAR=VALUE_B
# (each its own rocprofv3 --kernel-trace --stats run; rocprofv3 runs python directly).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for kv in "$@"; do
  i=$((i+1))
  export "${kv?}"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/ab_$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 12 --warmup 3 > "$ROOT/gpurun_out/ab_$i.log" 2>&1 || exit $?
  python3 "$ROOT/scripts/prof_summary.py" "$ROOT"/gpurun_out/ab_$i/*results.db > "$ROOT/gpurun_out/ab_$i.md" 2>&1 || \
    python3 "$ROOT/scripts/prof_summary.py" "$ROOT"/gpurun_out/ab_$i/*/*results.db > "$ROOT/gpurun_out/ab_$i.md"
done
