#!/bin/bash
# Round 3: list-window arena on the GPU (tests + config 8), full GPU suite, headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r3h_tests.log 2>&1 || { tail -60 gpurun_out/r3h_tests.log; exit 1; }
tail -2 gpurun_out/r3h_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 8 > gpurun_out/r3h_cfg8.json 2> gpurun_out/r3h_cfg8.err || { tail -30 gpurun_out/r3h_cfg8.err; exit 1; }
cat gpurun_out/r3h_cfg8.json
timeout -k 10 300 python -u bench.py > gpurun_out/r3h_bench.json 2> gpurun_out/r3h_bench.err || { tail -30 gpurun_out/r3h_bench.err; exit 1; }
cat gpurun_out/r3h_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3h_prof8 -o cfg8 -- python3 -m mxstream.models.bench_configs --config 8 --steps 12 > gpurun_out/r3h_rocprof8.log 2>&1 || { tail -30 gpurun_out/r3h_rocprof8.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3h_prof8 --width 90 > gpurun_out/r3h_kernels8.md && head -16 gpurun_out/r3h_kernels8.md
