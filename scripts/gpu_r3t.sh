#!/bin/bash
# Round 3: sparse pane rows + exact LDS plan in window_agg, session insert counting fix.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_sessions.py tests/test_loopback.py tests/test_window_operator_cpu.py > gpurun_out/r3t_tests.log 2>&1 || { tail -30 gpurun_out/r3t_tests.log; exit 1; }
tail -1 gpurun_out/r3t_tests.log
for sp in 1 0; do
  MXS_SPARSE_PANES=$sp timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3t_cfg4_s$sp.log 2>&1 || { tail -20 gpurun_out/r3t_cfg4_s$sp.log; exit 1; }
  tail -1 gpurun_out/r3t_cfg4_s$sp.log
done
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/r3t_bench.log 2>&1 || { tail -20 gpurun_out/r3t_bench.log; exit 1; }
tail -1 gpurun_out/r3t_bench.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3t_cfg5.log 2>&1 || { tail -20 gpurun_out/r3t_cfg5.log; exit 1; }
tail -1 gpurun_out/r3t_cfg5.log
MXS_SESS_SUB_LOG2=11 timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3t_cfg5_sub11.log 2>&1 || { tail -20 gpurun_out/r3t_cfg5_sub11.log; exit 1; }
tail -1 gpurun_out/r3t_cfg5_sub11.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 10 > gpurun_out/r3t_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3t_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3t_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3t_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3t_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3t_prof4.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3t_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 5 > "$ROOT/gpurun_out/r3t_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3t_prof5.log"; exit 1; }
echo done
