#!/bin/bash
# Round 3: GPU tests of the new paths, config 7 (BandwidthMonitorWithEventTime through the
# DataStream API, device ingest) with a host cProfile, and the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ingest.py tests/test_loopback.py tests/test_checkpoint.py tests/test_api_gpu.py tests/test_datastream_device_exchange.py > gpurun_out/r3b_tests.log 2>&1 || { tail -50 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 > gpurun_out/r3b_cfg7.json 2> gpurun_out/r3b_cfg7.err || { tail -30 gpurun_out/r3b_cfg7.err; exit 1; }
cat gpurun_out/r3b_cfg7.json
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 7 --profile > gpurun_out/r3b_cfg7_prof.txt 2>&1 || { tail -30 gpurun_out/r3b_cfg7_prof.txt; exit 1; }
head -75 gpurun_out/r3b_cfg7_prof.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || { tail -30 gpurun_out/r3b_bench.err; exit 1; }
cat gpurun_out/r3b_bench.json
