#!/bin/bash
# Round 3: fused re-firing + session single-wait fold -- GPU tests, config 4, config 5 (+ A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_sessions.py > gpurun_out/r3s_tests.log 2>&1 || { tail -30 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
for fz in 1 0; do
  MXS_FUSED_REFIRE=$fz timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3s_cfg4_f$fz.log 2>&1 || { tail -20 gpurun_out/r3s_cfg4_f$fz.log; exit 1; }
  tail -1 gpurun_out/r3s_cfg4_f$fz.log
done
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3s_cfg5.log 2>&1 || { tail -20 gpurun_out/r3s_cfg5.log; exit 1; }
tail -1 gpurun_out/r3s_cfg5.log
MXS_SESS_SUB_LOG2=11 timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3s_cfg5_sub11.log 2>&1 || { tail -20 gpurun_out/r3s_cfg5_sub11.log; exit 1; }
tail -1 gpurun_out/r3s_cfg5_sub11.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 10 > gpurun_out/r3s_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3s_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3s_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3s_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3s_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3s_prof4.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3s_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 5 > "$ROOT/gpurun_out/r3s_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3s_prof5.log"; exit 1; }
echo done
