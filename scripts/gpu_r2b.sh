#!/bin/bash
# Round-2 GPU check 2: GPU tests after the device-index fix, headline bench (serial at G=1),
# kernel tables of the G=8 loopback step (pipelined and serial).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loop8 -o loop8 -- python3 scripts/loopback_bench.py --world 8 --steps 6 --warmup 2 --no-pipeline --out gpurun_out/loop8_nopipe.json > gpurun_out/prof_loop8.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_loop8p -o loop8p -- python3 scripts/loopback_bench.py --world 8 --steps 6 --warmup 2 --out gpurun_out/loop8_pipe.json > gpurun_out/prof_loop8p.log 2>&1
echo "exit $?"
