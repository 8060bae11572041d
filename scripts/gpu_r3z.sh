#!/bin/bash
# Round 3: session fold (register-held values, overlapped host fire) -- tests, config 5 (+revisit), profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_sessions.py tests/test_loopback.py tests/test_checkpoint.py tests/test_state_guards.py -k "session or Session" \
  > gpurun_out/r3z_tests.log 2>&1 || { tail -30 gpurun_out/r3z_tests.log; exit 1; }
tail -1 gpurun_out/r3z_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 10 > gpurun_out/r3z_cfg5.log 2>&1 || { tail -20 gpurun_out/r3z_cfg5.log; exit 1; }
tail -1 gpurun_out/r3z_cfg5.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3z_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3z_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3z_cfg5r.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3z_prof5" -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 --warmup 10 > "$ROOT/gpurun_out/r3z_prof5.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3z_prof5.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3z_prof5 --steps 20 --busy 400 > gpurun_out/r3z_prof5.md
echo done
