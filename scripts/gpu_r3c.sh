#!/bin/bash
# Round 3: config 7 after fire-kernel ILP / adaptive dense state / H2D prefetch; kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ingest.py tests/test_api_gpu.py tests/test_columnar_ingest.py tests/test_datastream_device_exchange.py > gpurun_out/r3c_tests.log 2>&1 || { tail -50 gpurun_out/r3c_tests.log; exit 1; }
tail -2 gpurun_out/r3c_tests.log
for b in 1048576 4194304; do
  timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --batch $b > gpurun_out/r3c_cfg7_b$b.json 2> gpurun_out/r3c_cfg7.err || { tail -30 gpurun_out/r3c_cfg7.err; exit 1; }
  cat gpurun_out/r3c_cfg7_b$b.json
done
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --profile > gpurun_out/r3c_cfg7_prof.txt 2>&1 || { tail -30 gpurun_out/r3c_cfg7_prof.txt; exit 1; }
head -50 gpurun_out/r3c_cfg7_prof.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3c_prof -o cfg7 -- python3 -m mxstream.models.bench_configs --config 7 > $GRAFT_REPO_ROOT/gpurun_out/r3c_rocprof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3c_rocprof.log; exit 1; }
cd $GRAFT_REPO_ROOT && find gpurun_out/r3c_prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/r3c_prof -name "*kernel_stats.csv" | head -1); head -25 "$f"
