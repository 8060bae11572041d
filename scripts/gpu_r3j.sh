#!/bin/bash
# Round 3: config 4 with the host-DRAM tier (key space outgrowing HBM), spill GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_window_operator_cpu.py tests/test_checkpoint.py tests/test_sessions.py tests/test_api_gpu.py > gpurun_out/r3j_tests.log 2>&1 || { tail -60 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
timeout -k 10 400 python -u -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 60 > gpurun_out/r3j_cfg4s.json 2> gpurun_out/r3j_cfg4s.err || { tail -30 gpurun_out/r3j_cfg4s.err; exit 1; }
cat gpurun_out/r3j_cfg4s.json
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3j_cfg5.json 2> gpurun_out/r3j_cfg5.err || { tail -30 gpurun_out/r3j_cfg5.err; exit 1; }
cat gpurun_out/r3j_cfg5.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3j_prof5 -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 > gpurun_out/r3j_rocprof5.log 2>&1 || { tail -30 gpurun_out/r3j_rocprof5.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3j_prof5 --width 90 > gpurun_out/r3j_kernels5.md && head -12 gpurun_out/r3j_kernels5.md
