#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 2 --steps 20 --warmup 5 > gpurun_out/cfg2.log 2>&1 &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench.log 2>&1
