#!/bin/bash
# GPU tests (all), G=1 serial headline profile (kernel trace) and the host-side stage trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python bench.py --steps 24 --warmup 6 --trace gpurun_out/bench_trace.json > gpurun_out/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g1 -o g1 -- python3 bench.py --steps 12 --warmup 4 > gpurun_out/prof_g1.log 2>&1
echo "exit $?"
