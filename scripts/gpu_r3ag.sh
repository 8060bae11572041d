#!/bin/bash
# Round 3: rolling-state spill tier (tests + config 2 spill bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rolling.py > gpurun_out/r3ag_tests.log 2>&1 || { tail -30 gpurun_out/r3ag_tests.log; exit 1; }
tail -1 gpurun_out/r3ag_tests.log
timeout -k 10 400 python -m mxstream.models.bench_configs --config 2 --spill --steps 20 --warmup 30 > gpurun_out/r3ag_cfg2s.log 2>&1 || { tail -20 gpurun_out/r3ag_cfg2s.log; exit 1; }
tail -1 gpurun_out/r3ag_cfg2s.log
