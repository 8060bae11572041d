#!/bin/bash
# Round 3: async idle eviction (sessions) + radix scatter with register-held destinations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sort.py tests/test_sessions.py tests/test_rolling.py tests/test_gpu_kernels.py -k "sort or session or Session or rolling or median" > gpurun_out/r3ai_tests.log 2>&1 || { tail -30 gpurun_out/r3ai_tests.log; exit 1; }
tail -1 gpurun_out/r3ai_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3ai_cfg5.log 2>&1 || { tail -20 gpurun_out/r3ai_cfg5.log; exit 1; }
tail -1 gpurun_out/r3ai_cfg5.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3ai_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3ai_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3ai_cfg5r.log
timeout -k 10 200 python -m mxstream.models.bench_configs --config 2 --hashed-keys --sort-path --keys 1000000 --steps 20 --warmup 5 > gpurun_out/r3ai_cfg2_sort1m.log 2>&1 || { tail -20 gpurun_out/r3ai_cfg2_sort1m.log; exit 1; }
tail -1 gpurun_out/r3ai_cfg2_sort1m.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3ai_prof2" -o cfg2 -- python3 -m mxstream.models.bench_configs --config 2 --hashed-keys --sort-path --keys 1000000 --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/r3ai_prof2.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
python scripts/rocpd_summary.py gpurun_out/r3ai_prof2 --steps 13 > gpurun_out/r3ai_prof2.md
head -8 gpurun_out/r3ai_prof2.md
