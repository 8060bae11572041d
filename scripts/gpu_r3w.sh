#!/bin/bash
# Round 3: dirty-pane mask in the fused re-firing; config 4; loopback G=8 records profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py > gpurun_out/r3w_tests.log 2>&1 || { tail -30 gpurun_out/r3w_tests.log; exit 1; }
tail -1 gpurun_out/r3w_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3w_cfg4.log 2>&1 || { tail -20 gpurun_out/r3w_cfg4.log; exit 1; }
tail -1 gpurun_out/r3w_cfg4.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3w_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3w_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3w_prof4.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3w_proflb" -o lb -- python3 "$ROOT/scripts/loopback_bench.py" --world 8 --steps 6 --warmup 3 --exchange records --out "$ROOT/gpurun_out/r3w_lb.json" > "$ROOT/gpurun_out/r3w_proflb.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3w_proflb.log"; exit 1; }
echo done
