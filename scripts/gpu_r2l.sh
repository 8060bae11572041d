#!/bin/bash
# GPU text ingest with the native line-start kernels: parse/ingest GPU tests, config 1 GPU path,
# kernel table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_text_gpu.py tests/test_columnar_ingest.py tests/test_filter_compact.py tests/test_api_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_text.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 20 --warmup 3 > gpurun_out/cfg1_gpu.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1b -o run -- python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 20 --warmup 3 > gpurun_out/cfg1_prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
