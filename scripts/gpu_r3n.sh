#!/bin/bash
# Round 3: narrow records beyond 512 buckets (config 4), GPU window tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_loopback.py tests/test_api_gpu.py > gpurun_out/r3n_tests.log 2>&1 || { tail -60 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 4 > gpurun_out/r3n_cfg4.json 2> gpurun_out/r3n_cfg4.err || { tail -30 gpurun_out/r3n_cfg4.err; exit 1; }
cat gpurun_out/r3n_cfg4.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3n_prof4 -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 > gpurun_out/r3n_rocprof4.log 2>&1 || { tail -30 gpurun_out/r3n_rocprof4.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3n_prof4 --width 90 --steps 42 > gpurun_out/r3n_kernels4.md && head -12 gpurun_out/r3n_kernels4.md
