#!/bin/bash
# Filter compaction on the GPU: numerics vs NumPy, config 1 GPU path (parse + compaction + alert
# gather), kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_filter_compact.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_filter.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 20 --warmup 3 > gpurun_out/cfg1_gpu.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 20 --warmup 3 > gpurun_out/cfg1_prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
