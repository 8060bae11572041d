#!/bin/bash
# A/B of the window_agg records-per-thread (interleaved probes) + kernel stats of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench_u8.log 2>&1 &&
MXS_AGG_U=4 timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench_u4.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench_u8b.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 12 --warmup 3 > "$ROOT/gpurun_out/prof.log" 2>&1
