#!/bin/bash
# Round 3: session fold launched behind the partition (one host wait), counter-based occupancy,
# counted fire copy -- session GPU tests, config 5 / 5r, and the config 5 kernel timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_sessions.py tests/test_gpu_kernels.py > gpurun_out/r3r_tests.log 2>&1 || { tail -30 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3r_cfg5.log 2>&1 || { tail -20 gpurun_out/r3r_cfg5.log; exit 1; }
tail -1 gpurun_out/r3r_cfg5.log
MXS_SESS_SUB_LOG2=11 timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3r_cfg5_sub11.log 2>&1 || { tail -20 gpurun_out/r3r_cfg5_sub11.log; exit 1; }
tail -1 gpurun_out/r3r_cfg5_sub11.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 10 > gpurun_out/r3r_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3r_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3r_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3r_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 5 > "$ROOT/gpurun_out/r3r_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3r_prof5.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3r_prof5 --steps 15 --busy 300 > gpurun_out/r3r_prof5_summary.md 2>&1
tail -25 gpurun_out/r3r_prof5_summary.md
