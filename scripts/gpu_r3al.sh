#!/bin/bash
# Round 3: headline kernel table from the final tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3al_profh" -o head -- python3 "$ROOT/bench.py" --steps 24 --warmup 6 --latency-firings 0 --no-hashed-figure > "$ROOT/gpurun_out/r3al_profh.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3al_profh.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3al_profh --steps 30 > gpurun_out/r3al_profh.md
head -14 gpurun_out/r3al_profh.md
tail -1 gpurun_out/r3al_profh.log | cut -c1-200
