#!/bin/bash
# Round 3: config 5 session sub-table size A/B (4096 vs 2048 vs 1024 slots per fold workgroup).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
for L in 0 11 10; do
  MXS_SESS_SUB_LOG2=$L timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3l_cfg5_$L.json 2> gpurun_out/r3l_cfg5.err || { tail -30 gpurun_out/r3l_cfg5.err; exit 1; }
  cat gpurun_out/r3l_cfg5_$L.json
done
MXS_SESS_SUB_LOG2=11 timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3l_prof5 -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 > gpurun_out/r3l_rocprof5.log 2>&1 || { tail -30 gpurun_out/r3l_rocprof5.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3l_prof5 --width 90 > gpurun_out/r3l_kernels5.md && head -10 gpurun_out/r3l_kernels5.md
