#!/bin/bash
# Round 4: PMC passes over loopback G = 8 records exchange (partition with 8 destinations, sender-side combiner).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONPATH=$ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc $set \
    -d "$ROOT/gpurun_out/pmc_r4_lb8_$i" -o run -- python3 "$ROOT/scripts/loopback_bench.py" --world 8 --exchange records --steps 3 --warmup 1 > "$ROOT/gpurun_out/pmc_r4_lb8_$i.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/pmc_r4_lb8_$i.log"; exit 1; }
done
cd "$ROOT"
python scripts/pmc_summary.py "gpurun_out/pmc_r4_lb8_*/**/*counter_collection.csv" > gpurun_out/pmc_r4_lb8.md
cat gpurun_out/pmc_r4_lb8.md | head -80
