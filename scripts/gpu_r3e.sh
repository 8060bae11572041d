#!/bin/bash
# Round 3: batched multi-window fire kernel + columnar print path; GPU tests, config 7, kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_api_gpu.py tests/test_ingest.py tests/test_datastream_device_exchange.py \
  tests/test_loopback.py tests/test_checkpoint.py tests/test_sessions.py > gpurun_out/r3e_tests.log 2>&1 || { tail -50 gpurun_out/r3e_tests.log; exit 1; }
tail -2 gpurun_out/r3e_tests.log
for b in 1048576 4194304; do
  timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --batch $b > gpurun_out/r3e_cfg7_b$b.json 2> gpurun_out/r3e_cfg7.err || { tail -30 gpurun_out/r3e_cfg7.err; exit 1; }
  cat gpurun_out/r3e_cfg7_b$b.json
done
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --profile > gpurun_out/r3e_cfg7_prof.txt 2>&1 || { tail -30 gpurun_out/r3e_cfg7_prof.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3e_prof -o cfg7 -- python3 -m mxstream.models.bench_configs --config 7 > gpurun_out/r3e_rocprof.log 2>&1 || { tail -30 gpurun_out/r3e_rocprof.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3e_prof --width 90 > gpurun_out/r3e_kernels.md && head -30 gpurun_out/r3e_kernels.md
