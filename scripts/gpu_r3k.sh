#!/bin/bash
# Round 3: PMC counters of the config 5 session fold (lookup-sort kernel) -- two passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3k_pmc1 -o p1 -- python3 -m mxstream.models.bench_configs --config 5 --steps 3 --warmup 2 > gpurun_out/r3k_pmc1.log 2>&1 || { tail -20 gpurun_out/r3k_pmc1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3k_pmc2 -o p2 -- python3 -m mxstream.models.bench_configs --config 5 --steps 3 --warmup 2 > gpurun_out/r3k_pmc2.log 2>&1 || { tail -20 gpurun_out/r3k_pmc2.log; exit 1; }
python3 scripts/pmc_summary.py "gpurun_out/r3k_pmc1/**/*counter_collection.csv" "gpurun_out/r3k_pmc2/**/*counter_collection.csv" > gpurun_out/r3k_pmc.md; grep -A16 "session_lookup_sort\|session_merge_small" gpurun_out/r3k_pmc.md | head -60
