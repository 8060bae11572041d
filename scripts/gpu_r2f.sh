#!/bin/bash
# Re-validation of HEAD on a fresh box: GPU tests, smoke, headline bench, kernel table, config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
test -f mxstream/_mxs_native*.so &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python bench.py --zipf 1.2 > gpurun_out/bench_zipf.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 24 --warmup 6 > gpurun_out/bench_prof.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 2 --steps 20 --warmup 5 > gpurun_out/cfg2.log 2>&1 &&
timeout -k 10 300 python scripts/loopback_bench.py --world 8 > gpurun_out/loop8.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
