#!/bin/bash
# Round 3: two-level partition (> 512 buckets), sparse pane rows, exact window_agg LDS plan,
# session insert counting -- GPU tests, config 4 A/Bs, headline, config 5, profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_sessions.py tests/test_loopback.py > gpurun_out/r3u_tests.log 2>&1 || { tail -30 gpurun_out/r3u_tests.log; exit 1; }
tail -1 gpurun_out/r3u_tests.log
for v in "1 1" "0 1" "1 0"; do
  set -- $v
  MXS_TWO_LEVEL=$1 MXS_SPARSE_PANES=$2 timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3u_cfg4_t$1s$2.log 2>&1 || { tail -20 gpurun_out/r3u_cfg4_t$1s$2.log; exit 1; }
  echo "two_level=$1 sparse=$2: $(tail -1 gpurun_out/r3u_cfg4_t$1s$2.log)"
done
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/r3u_bench.log 2>&1 || { tail -20 gpurun_out/r3u_bench.log; exit 1; }
tail -1 gpurun_out/r3u_bench.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3u_cfg5.log 2>&1 || { tail -20 gpurun_out/r3u_cfg5.log; exit 1; }
tail -1 gpurun_out/r3u_cfg5.log
MXS_SESS_SUB_LOG2=11 timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3u_cfg5_sub11.log 2>&1 || { tail -20 gpurun_out/r3u_cfg5_sub11.log; exit 1; }
tail -1 gpurun_out/r3u_cfg5_sub11.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 10 > gpurun_out/r3u_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3u_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3u_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3u_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3u_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3u_prof4.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3u_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 5 > "$ROOT/gpurun_out/r3u_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3u_prof5.log"; exit 1; }
echo done
