#!/bin/bash
# Round 3: config 5 with revisits (radix-indexed cold chunks); loopback G=8 records-exchange profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "spill or compact or tier" > gpurun_out/r3aa_tests.log 2>&1 || { tail -30 gpurun_out/r3aa_tests.log; exit 1; }
tail -1 gpurun_out/r3aa_tests.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --spill --steps 6 --warmup 6 > gpurun_out/r3aa_cfg4s.log 2>&1 || { tail -20 gpurun_out/r3aa_cfg4s.log; exit 1; }
tail -1 gpurun_out/r3aa_cfg4s.log
timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --revisit 0.01 --steps 20 --warmup 14 > gpurun_out/r3aa_cfg5r.log 2>&1 || { tail -20 gpurun_out/r3aa_cfg5r.log; exit 1; }
tail -1 gpurun_out/r3aa_cfg5r.log
timeout -k 10 300 python scripts/loopback_bench.py --world 8 --steps 12 --warmup 4 --exchange records --out gpurun_out/r3aa_lb.json > gpurun_out/r3aa_lb.log 2>&1 || { tail -20 gpurun_out/r3aa_lb.log; exit 1; }
cat gpurun_out/r3aa_lb.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r3aa_proflb" -o lb -- python3 "$ROOT/scripts/loopback_bench.py" --world 8 --steps 6 --warmup 3 --exchange records --out "$ROOT/gpurun_out/r3aa_lbp.json" > "$ROOT/gpurun_out/r3aa_proflb.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/r3aa_proflb.log"; exit 1; }
cd "$ROOT"
python scripts/rocpd_summary.py gpurun_out/r3aa_proflb --steps 9 --busy 600 > gpurun_out/r3aa_proflb.md
echo done
