#!/bin/bash
# Round 3: side-stream fired-row copies, lazily resolved fused re-firing -- tests + config 4 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_loopback.py tests/test_sessions.py > gpurun_out/r3v_tests.log 2>&1 || { tail -30 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
for cs in 1 0; do
  MXS_COPY_STREAM=$cs timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3v_cfg4_cs$cs.log 2>&1 || { tail -20 gpurun_out/r3v_cfg4_cs$cs.log; exit 1; }
  echo "copy_stream=$cs: $(tail -1 gpurun_out/r3v_cfg4_cs$cs.log)"
done
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/r3v_bench.log 2>&1 || { tail -20 gpurun_out/r3v_bench.log; exit 1; }
tail -1 gpurun_out/r3v_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3v_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3v_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3v_prof4.log"; exit 1; }
echo done
