#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -m pytest tests/test_rolling.py tests/test_sessions.py -m gpu -x -q > gpurun_out/pytest_rolling.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 2 --steps 20 --warmup 5 > gpurun_out/cfg2.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cfg2" -o cfg2 -- python3 -m mxstream.models.bench_configs --config 2 --steps 8 --warmup 4 > "$GRAFT_REPO_ROOT/gpurun_out/cfg2_prof.log" 2>&1
