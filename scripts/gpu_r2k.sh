#!/bin/bash
# Config 4 fired-row D2H A/B: copy kernel into the mapped pinned slab (default) vs SDMA
# hipMemcpyAsync (MXS_D2H=dma), twice each, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 32 > gpurun_out/cfg4_kernel_$i.log 2>&1 || exit $?
  MXS_D2H=dma timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 32 > gpurun_out/cfg4_dma_$i.log 2>&1 || exit $?
done
echo "exit 0"
