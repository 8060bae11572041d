#!/bin/bash
# Round 3: async firing (device-counted row copy, lazy resolution) -- tests, config 4, headline,
# config 4 kernel timeline (busy/idle).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_loopback.py > gpurun_out/r3q_tests.log 2>&1 || { tail -30 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
for af in 0 1; do
  MXS_ASYNC_FIRE=$af timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3q_cfg4_af$af.log 2>&1 || { tail -20 gpurun_out/r3q_cfg4_af$af.log; exit 1; }
  tail -1 gpurun_out/r3q_cfg4_af$af.log
done
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/r3q_bench.log 2>&1 || { tail -20 gpurun_out/r3q_bench.log; exit 1; }
tail -1 gpurun_out/r3q_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3q_prof4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/r3q_prof4.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3q_prof4.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3q_prof4 --steps 42 --busy 400 > gpurun_out/r3q_prof4_summary.md 2>&1
tail -25 gpurun_out/r3q_prof4_summary.md
