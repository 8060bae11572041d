#!/bin/bash
# Round 3: config 4 kernel table after batched firing / compact rows / grouped loads; D2H A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 4 > gpurun_out/r3m_cfg4.json 2> gpurun_out/r3m_cfg4.err || { tail -30 gpurun_out/r3m_cfg4.err; exit 1; }
cat gpurun_out/r3m_cfg4.json
MXS_D2H=dma timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 4 > gpurun_out/r3m_cfg4_dma.json 2> gpurun_out/r3m_cfg4.err || { tail -30 gpurun_out/r3m_cfg4.err; exit 1; }
cat gpurun_out/r3m_cfg4_dma.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3m_prof4 -o cfg4 -- python3 -m mxstream.models.bench_configs --config 4 --steps 10 > gpurun_out/r3m_rocprof4.log 2>&1 || { tail -30 gpurun_out/r3m_rocprof4.log; exit 1; }
python3 scripts/rocpd_summary.py gpurun_out/r3m_prof4 --width 90 --steps 42 > gpurun_out/r3m_kernels4.md && head -14 gpurun_out/r3m_kernels4.md
timeout -k 10 300 python -u -m mxstream.models.bench_configs --config 5 > gpurun_out/r3m_cfg5.json 2> gpurun_out/r3m_cfg5.err || { tail -30 gpurun_out/r3m_cfg5.err; exit 1; }
cat gpurun_out/r3m_cfg5.json
