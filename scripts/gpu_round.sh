#!/bin/bash
# Full validation: build, all GPU tests, smoke, headline bench, configs 1 (CPU + GPU parse), 2, 4, 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --steps 10 --warmup 2 > gpurun_out/cfg1.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 10 --warmup 2 > gpurun_out/cfg1_gpu.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 2 --steps 20 --warmup 5 > gpurun_out/cfg2.log 2>&1 &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/cfg5.log 2>&1
[ $? -eq 0 ] && timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 14 > gpurun_out/cfg6.log 2>&1
