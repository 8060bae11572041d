#!/bin/bash
# Round 3: config 4 spill (threaded tier merge + C++ epilogue), config 5 / 5r (dense extract).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_sessions.py -k "spill or compact or tier or session or Session" > gpurun_out/r3ad_tests.log 2>&1 || { tail -30 gpurun_out/r3ad_tests.log; exit 1; }
tail -1 gpurun_out/r3ad_tests.log
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3ad_cfg4s.log 2>&1 || { tail -20 gpurun_out/r3ad_cfg4s.log; exit 1; }
tail -1 gpurun_out/r3ad_cfg4s.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3ad_cfg5.log 2>&1 || { tail -20 gpurun_out/r3ad_cfg5.log; exit 1; }
tail -1 gpurun_out/r3ad_cfg5.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3ad_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3ad_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3ad_cfg5r.log
timeout -k 10 400 python -m cProfile -s tottime -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3ad_cfg4s_cprof.log 2>&1 || { tail -20 gpurun_out/r3ad_cfg4s_cprof.log; exit 1; }
head -30 gpurun_out/r3ad_cfg4s_cprof.log | tail -22
