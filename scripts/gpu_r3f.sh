#!/bin/bash
# Round 3: config 5 (sessions + spill) and config 4 baselines with kernel tables before the rework.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3f_cfg5.json 2> gpurun_out/r3f_cfg5.err || { tail -30 gpurun_out/r3f_cfg5.err; exit 1; }
cat gpurun_out/r3f_cfg5.json
MXS_SESSION_SORT=radix timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3f_cfg5_radix.json 2> gpurun_out/r3f_cfg5.err || { tail -30 gpurun_out/r3f_cfg5.err; exit 1; }
cat gpurun_out/r3f_cfg5_radix.json
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 --revisit 0.01 > gpurun_out/r3f_cfg5r.json 2> gpurun_out/r3f_cfg5r.err || { tail -30 gpurun_out/r3f_cfg5r.err; exit 1; }
cat gpurun_out/r3f_cfg5r.json
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 4 > gpurun_out/r3f_cfg4.json 2> gpurun_out/r3f_cfg4.err || { tail -30 gpurun_out/r3f_cfg4.err; exit 1; }
cat gpurun_out/r3f_cfg4.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3f_prof5 -o cfg5 -- python3 -m mxstream.models.bench_configs --config 5 --steps 10 > gpurun_out/r3f_rocprof5.log 2>&1 || { tail -30 gpurun_out/r3f_rocprof5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3f_prof4 -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 > gpurun_out/r3f_rocprof4.log 2>&1 || { tail -30 gpurun_out/r3f_rocprof4.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3f_prof5 --width 90 > gpurun_out/r3f_kernels5.md && head -25 gpurun_out/r3f_kernels5.md
python3 scripts/rocpd_summary.py gpurun_out/r3f_prof4 --width 90 > gpurun_out/r3f_kernels4.md && head -25 gpurun_out/r3f_kernels4.md
