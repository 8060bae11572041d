#!/bin/bash
# Round 3: ranked list-window firing on the GPU (tests, config 8 + kernel table).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_list_window.py tests/test_api_gpu.py tests/test_gpu_kernels.py > gpurun_out/r3i_tests.log 2>&1 || { tail -60 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 8 > gpurun_out/r3i_cfg8.json 2> gpurun_out/r3i_cfg8.err || { tail -30 gpurun_out/r3i_cfg8.err; exit 1; }
cat gpurun_out/r3i_cfg8.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3i_prof8 -o cfg8 -- python3 -m mxstream.models.bench_configs --config 8 --steps 12 > gpurun_out/r3i_rocprof8.log 2>&1 || { tail -30 gpurun_out/r3i_rocprof8.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3i_prof8 --width 90 > gpurun_out/r3i_kernels8.md && head -16 gpurun_out/r3i_kernels8.md
