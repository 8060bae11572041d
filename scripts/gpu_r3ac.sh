#!/bin/bash
# Round 3: config 4 spill variant after the parallel tiered firing; host profile of the same.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3ac_cfg4s.log 2>&1 || { tail -20 gpurun_out/r3ac_cfg4s.log; exit 1; }
tail -1 gpurun_out/r3ac_cfg4s.log
timeout -k 10 400 python -m cProfile -s tottime -m mxstream.models.bench_configs --config 4 --spill --steps 30 --warmup 40 > gpurun_out/r3ac_cfg4s_cprof.log 2>&1 || { tail -20 gpurun_out/r3ac_cfg4s_cprof.log; exit 1; }
head -45 gpurun_out/r3ac_cfg4s_cprof.log | tail -38
