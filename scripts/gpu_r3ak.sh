#!/bin/bash
# Round 3: host profile of config 5 (main thread).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -m cProfile -s tottime -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3ak_cfg5_cprof.log 2>&1 || { tail -20 gpurun_out/r3ak_cfg5_cprof.log; exit 1; }
head -40 gpurun_out/r3ak_cfg5_cprof.log
