#!/bin/bash
# Session-window GPU checks + config 5 bench + kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -m pytest tests/test_sessions.py -m gpu -x -q > gpurun_out/pytest_sessions.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/cfg5.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 8 --warmup 6 > "$GRAFT_REPO_ROOT/gpurun_out/cfg5_prof.log" 2>&1
