#!/bin/bash
# Round 3 closing validation: all GPU tests, smoke, headline bench, configs 2/4/5 (+ spill variants), 6.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ah_pytest.log 2>&1 || { tail -30 gpurun_out/r3ah_pytest.log; exit 1; }
tail -1 gpurun_out/r3ah_pytest.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ah_smoke.log 2>&1 || { tail -20 gpurun_out/r3ah_smoke.log; exit 1; }
tail -1 gpurun_out/r3ah_smoke.log
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/r3ah_bench.log 2>&1 || { tail -20 gpurun_out/r3ah_bench.log; exit 1; }
tail -1 gpurun_out/r3ah_bench.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 2 --steps 20 --warmup 5 > gpurun_out/r3ah_cfg2.log 2>&1 && tail -1 gpurun_out/r3ah_cfg2.log &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 2 --spill --steps 20 --warmup 30 > gpurun_out/r3ah_cfg2s.log 2>&1 && tail -1 gpurun_out/r3ah_cfg2s.log &&
timeout -k 10 400 python -m mxstream.models.bench_configs --config 4 --steps 30 --warmup 30 > gpurun_out/r3ah_cfg4.log 2>&1 && tail -1 gpurun_out/r3ah_cfg4.log &&
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3ah_cfg5.log 2>&1 && tail -1 gpurun_out/r3ah_cfg5.log
