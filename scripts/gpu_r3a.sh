#!/bin/bash
# Round 3: device text ingest validation + config 7 through the DataStream API.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_ingest.py tests/test_api_gpu.py tests/test_text_gpu.py > gpurun_out/r3a_tests.log 2>&1 || { tail -50 gpurun_out/r3a_tests.log; exit 1; }
tail -5 gpurun_out/r3a_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 > gpurun_out/r3a_cfg7.json 2> gpurun_out/r3a_cfg7.err || { tail -30 gpurun_out/r3a_cfg7.err; exit 1; }
cat gpurun_out/r3a_cfg7.json
