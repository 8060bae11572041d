#!/bin/bash
# Vector-metric windows on the GPU: numerics tests, MFMA vs VALU bench, kernel stats, MFMA PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest tests/test_vector_window.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/vec_tests.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 14 > gpurun_out/cfg6_mfma.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 14 --valu > gpurun_out/cfg6_valu.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 14 --dim 128 > gpurun_out/cfg6_d128.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_vec" -o run -- \
  python3 -m mxstream.models.bench_configs --config 6 --steps 6 --warmup 14 > "$ROOT/gpurun_out/prof_vec.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$ROOT/gpurun_out/pmc_vec" -o run --output-format csv -- \
  python3 -m mxstream.models.bench_configs --config 6 --steps 3 --warmup 14 > "$ROOT/gpurun_out/pmc_vec.log" 2>&1
