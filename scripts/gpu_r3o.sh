#!/bin/bash
# Round 3: records exchange without the combiner host wait -- loopback GPU tests + G=8 per-rank step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
for ex in records partials; do
  timeout -k 10 300 python -u scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 --exchange $ex --out gpurun_out/r3o_lb8_$ex.json > gpurun_out/r3o_lb8_$ex.log 2>&1 || { tail -30 gpurun_out/r3o_lb8_$ex.log; exit 1; }
  tail -1 gpurun_out/r3o_lb8_$ex.log
done
