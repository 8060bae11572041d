#!/bin/bash
# PMC counter passes (each its own run, counters only with kernel-trace) on the kernel bench.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp
export KB_FILTER=${KB_FILTER:-partition} KB_ABLATE=${KB_ABLATE:-0} ROUNDS=${ROUNDS:-3}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT64" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU_INT32 SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc $set -d "$ROOT/gpurun_out/pmc$i" -o run -- \
    python3 "$ROOT/scripts/kbench.py" > "$ROOT/gpurun_out/pmc$i.log" 2>&1 || exit $?
done
