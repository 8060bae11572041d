#!/bin/bash
# Session promotion after the slot-insert fix: GPU session + C ABI tests, config 5 (+ revisits,
# promotion vs host fold), kernel table of the revisit run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sessions.py tests/test_capi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sessions.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/cfg5.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 14 --revisit 0.01 > gpurun_out/cfg5r.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5r -o run -- python -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 14 --revisit 0.01 > gpurun_out/cfg5r_prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
