#!/bin/bash
# Round 3: config 5 with the fused LDS sort (merge grid fixed), config 7 with a same-batch warm-up.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions.py tests/test_api_gpu.py tests/test_gpu_kernels.py > gpurun_out/r3g_tests.log 2>&1 || { tail -50 gpurun_out/r3g_tests.log; exit 1; }
tail -2 gpurun_out/r3g_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3g_cfg5.json 2> gpurun_out/r3g_cfg5.err || { tail -30 gpurun_out/r3g_cfg5.err; exit 1; }
cat gpurun_out/r3g_cfg5.json
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 --revisit 0.01 > gpurun_out/r3g_cfg5r.json 2> gpurun_out/r3g_cfg5r.err || { tail -30 gpurun_out/r3g_cfg5r.err; exit 1; }
cat gpurun_out/r3g_cfg5r.json
for b in 1048576 2097152 4194304; do
  timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --batch $b > gpurun_out/r3g_cfg7_b$b.json 2> gpurun_out/r3g_cfg7.err || { tail -30 gpurun_out/r3g_cfg7.err; exit 1; }
  cat gpurun_out/r3g_cfg7_b$b.json
done
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 4 > gpurun_out/r3g_cfg4.json 2> gpurun_out/r3g_cfg4.err || { tail -30 gpurun_out/r3g_cfg4.err; exit 1; }
cat gpurun_out/r3g_cfg4.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3g_prof5 -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 > gpurun_out/r3g_rocprof5.log 2>&1 || { tail -30 gpurun_out/r3g_rocprof5.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3g_prof5 --width 90 > gpurun_out/r3g_kernels5.md && head -16 gpurun_out/r3g_kernels5.md
