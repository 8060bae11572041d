#!/bin/bash
# Round-2 GPU check: GPU tests (loopback G>1 paths included), headline bench (pipelined),
# G=8 loopback per-rank step (pipelined and not), kernel stats of the headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench2.log 2>&1 &&
timeout -k 10 400 python scripts/loopback_bench.py --world 8 --steps 8 --warmup 3 --out gpurun_out/loop8.json > gpurun_out/loop8.log 2>&1 &&
timeout -k 10 400 python scripts/loopback_bench.py --world 8 --steps 8 --warmup 3 --no-pipeline --out gpurun_out/loop8_nopipe.json > gpurun_out/loop8_nopipe.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 12 --warmup 4 > gpurun_out/prof_bench.log 2>&1
echo "exit $?"
