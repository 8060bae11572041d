#!/bin/bash
# One GPU validation pass: gpu tests -> smoke -> short bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so trouble ends the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-24}
BATCH=${BATCH:-16777216}
test -f mxstream/_mxs_native*.so &&
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps $STEPS --warmup 6 --batch $BATCH > gpurun_out/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 12 --warmup 3 --batch $BATCH > "$ROOT/gpurun_out/prof.log" 2>&1
