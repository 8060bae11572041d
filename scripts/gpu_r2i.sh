#!/bin/bash
# Round-2 closing validation: every GPU test, smoke, headline bench, config 5 with revisits after
# the extract change, config 4 kernel table with the timed region dominating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 14 --revisit 0.01 > gpurun_out/cfg5r.log 2>&1 &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 32 > gpurun_out/cfg4.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o run -- python -m mxstream.models.bench_configs --config 4 --steps 40 --warmup 32 > gpurun_out/cfg4_prof.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
