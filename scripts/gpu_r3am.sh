#!/bin/bash
# Round 3: lazy tier purge -- spill GPU tests + config 4 spill.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_checkpoint.py -k "spill or compact or tier or window" > gpurun_out/r3am_tests.log 2>&1 || { tail -30 gpurun_out/r3am_tests.log; exit 1; }
tail -1 gpurun_out/r3am_tests.log
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3am_cfg4s.log 2>&1 || { tail -20 gpurun_out/r3am_cfg4s.log; exit 1; }
tail -1 gpurun_out/r3am_cfg4s.log
