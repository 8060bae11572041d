#!/bin/bash
# Round 3: kernel table of config 7 (device ingest) under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3d_prof -o cfg7 -- python3 -m mxstream.models.bench_configs --config 7 > gpurun_out/r3d_rocprof.log 2>&1 || { tail -30 gpurun_out/r3d_rocprof.log; exit 1; }
f=$(find gpurun_out/r3d_prof -name "*kernel_stats.csv" | head -1); echo "$f"; head -30 "$f"
