#!/bin/bash
# Round 3: config 4 spill variant (block-reserved window_compact output) + kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3ab_cfg4s.log 2>&1 || { tail -20 gpurun_out/r3ab_cfg4s.log; exit 1; }
tail -1 gpurun_out/r3ab_cfg4s.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3ab_prof4s" -o c4s -- python3 -m mxstream.models.bench_configs --config 4 --spill --steps 20 --warmup 40 > "$ROOT/gpurun_out/r3ab_prof4s.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3ab_prof4s.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3ab_prof4s --steps 60 --busy 800 > gpurun_out/r3ab_prof4s.md
echo done
