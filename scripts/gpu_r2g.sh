#!/bin/bash
# Session tier: GPU session tests (spill-set growth on the device, promotion of spilled keys back
# to HBM), config 5 with and without revisited spilled keys, promotion vs host fold.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sessions.py tests/test_state_guards.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sessions.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/cfg5.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 14 --revisit 0.01 > gpurun_out/cfg5r.log 2>&1 &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 14 --revisit 0.01 --host-fold > gpurun_out/cfg5r_host.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
