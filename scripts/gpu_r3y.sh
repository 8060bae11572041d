#!/bin/bash
# Round 3: hand-written radix sort (tests + rolling sort path) and a config 5 busy/idle timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sort.py tests/test_rolling.py tests/test_sessions.py tests/test_gpu_kernels.py -k "sort or rolling or median or count_window or session" \
  > gpurun_out/r3y_tests.log 2>&1 || { tail -30 gpurun_out/r3y_tests.log; exit 1; }
tail -1 gpurun_out/r3y_tests.log
timeout -k 10 200 python -m mxstream.models.bench_configs --config 2 --hashed-keys --sort-path --steps 20 --warmup 5 > gpurun_out/r3y_cfg2_sort10k.log 2>&1 || { tail -20 gpurun_out/r3y_cfg2_sort10k.log; exit 1; }
tail -1 gpurun_out/r3y_cfg2_sort10k.log
timeout -k 10 200 python -m mxstream.models.bench_configs --config 2 --hashed-keys --sort-path --keys 1000000 --steps 20 --warmup 5 > gpurun_out/r3y_cfg2_sort1m.log 2>&1 || { tail -20 gpurun_out/r3y_cfg2_sort1m.log; exit 1; }
tail -1 gpurun_out/r3y_cfg2_sort1m.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3y_cfg5.log 2>&1 || { tail -20 gpurun_out/r3y_cfg5.log; exit 1; }
tail -1 gpurun_out/r3y_cfg5.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3y_prof2" -o cfg2 -- python3 -m mxstream.models.bench_configs --config 2 --hashed-keys --sort-path --keys 1000000 --steps 10 --warmup 3 > "$ROOT/gpurun_out/r3y_prof2.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3y_prof2.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3y_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 10 > "$ROOT/gpurun_out/r3y_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3y_prof5.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3y_prof2 --steps 10 > gpurun_out/r3y_prof2.md
python scripts/rocpd_summary.py gpurun_out/r3y_prof5 --steps 10 --busy 400 > gpurun_out/r3y_prof5.md
echo done
