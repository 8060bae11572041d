#!/bin/bash
# Round 3: config 5 / 5r after the hot-key bitmaps in the host session store.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions.py > gpurun_out/r3af_tests.log 2>&1 || { tail -30 gpurun_out/r3af_tests.log; exit 1; }
tail -1 gpurun_out/r3af_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3af_cfg5.log 2>&1 || { tail -20 gpurun_out/r3af_cfg5.log; exit 1; }
tail -1 gpurun_out/r3af_cfg5.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3af_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3af_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3af_cfg5r.log
