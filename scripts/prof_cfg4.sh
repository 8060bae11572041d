#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out; export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_cfg4" -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 --warmup 25 > "$ROOT/gpurun_out/cfg4_prof.log" 2>&1
