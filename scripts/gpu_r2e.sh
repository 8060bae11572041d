#!/bin/bash
# Host-sync mode A/B of the G=1 headline (event vs stream sync, spin scheduling).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for mode in event stream; do
  MXS_SYNC=$mode timeout -k 10 200 python bench.py --steps 48 --warmup 8 > gpurun_out/bench_$mode.log 2>&1 || exit $?
  MXS_SPIN=1 MXS_SYNC=$mode timeout -k 10 200 python bench.py --steps 48 --warmup 8 > gpurun_out/bench_${mode}_spin.log 2>&1 || exit $?
done
MXS_SYNC=stream timeout -k 10 200 python bench.py --steps 48 --warmup 8 --trace gpurun_out/tr.json > gpurun_out/bench_stream_trace.log 2>&1
echo "exit $?"
