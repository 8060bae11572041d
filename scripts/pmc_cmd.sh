#!/bin/bash
# PMC counter passes (each its own run, counters only, with kernel-trace) over a Python module
# command, e.g.:  scripts/pmc_cmd.sh cfg5 mxstream.models.bench_configs --config 5 --steps 4 --warmup 4
# or a script under the repo root:  scripts/pmc_cmd.sh head bench.py --steps 6 --warmup 2
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG=$1; shift
export PYTHONPATH="$ROOT"
cd /tmp && export TMPDIR=/tmp
MOD=-m
if [[ $1 == *.py ]]; then MOD=""; set -- "$ROOT/$1" "${@:2}"; fi
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQC_TC_DATA_ATOMIC_REQ TA_BUFFER_ATOMIC_WAVEFRONTS_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc $set \
    -d "$ROOT/gpurun_out/pmc_${TAG}_$i" -o run -- python3 $MOD "$@" > "$ROOT/gpurun_out/pmc_${TAG}_$i.log" 2>&1 || exit $?
done
