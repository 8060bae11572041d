#!/bin/bash
# Round 3: lookup-sort probes the spill set once per newly claimed key.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sessions.py tests/test_loopback.py tests/test_checkpoint.py tests/test_state_guards.py tests/test_capi.py -k "session or Session" > gpurun_out/r3aj_tests.log 2>&1 || { tail -30 gpurun_out/r3aj_tests.log; exit 1; }
tail -1 gpurun_out/r3aj_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3aj_cfg5.log 2>&1 || { tail -20 gpurun_out/r3aj_cfg5.log; exit 1; }
tail -1 gpurun_out/r3aj_cfg5.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3aj_cfg5b.log 2>&1 && tail -1 gpurun_out/r3aj_cfg5b.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3aj_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3aj_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3aj_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3aj_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/r3aj_prof5.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
python scripts/rocpd_summary.py gpurun_out/r3aj_prof5 --steps 20 --busy 400 > gpurun_out/r3aj_prof5.md
python scripts/rocpd_summary.py gpurun_out/r3aj_prof5 --timeline 40 --width 45 | tail -40 > gpurun_out/r3aj_timeline.txt
head -6 gpurun_out/r3aj_prof5.md
