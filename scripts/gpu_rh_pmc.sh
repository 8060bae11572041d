#!/bin/bash
# PMC passes over the sort-free rolling COUNT (scripts/rolling_hist_ab.py, dense keys), one
# rocprofv3 run per counter set; csv under gpurun_out/<tag>/pmc<k>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-rh_pmc}; mkdir -p "$out"
export PYTHONPATH=$PWD DENSE=1
sets=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM")
k=0
for set in "${sets[@]}"; do
  k=$((k+1))
  (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
   timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $set -d "$out/pmc$k" -o run -- python3 scripts/rolling_hist_ab.py > "$out/pmc$k.log" 2>&1) || exit $?
done
echo done
