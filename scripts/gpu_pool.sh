#!/bin/bash
# Pinned slab pool for fired rows: GPU tests, headline bench x2, config 4 and 6, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pool_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/pool_bench_1.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/pool_bench_2.log 2>&1 &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/pool_cfg4.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 14 > gpurun_out/pool_cfg6.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/pool_prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 24 --warmup 3 > "$ROOT/gpurun_out/pool_prof.log" 2>&1
