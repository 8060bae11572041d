#!/bin/bash
# Local-global exchange: GPU tests, headline G=1, loopback G=8 (partials vs records) kernel tables.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so &&
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"
[ $st -eq 0 ] || [ $st -eq 1 ] || exit $st
timeout -k 10 300 python bench.py --steps 24 --warmup 6 > gpurun_out/bench.log 2>&1 &&
timeout -k 10 300 python scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 --out gpurun_out/loop8_partials.json > gpurun_out/loop8_partials.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lg8 -o lg8 -- python3 scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 --out gpurun_out/loop8_partials_prof.json > gpurun_out/prof_lg8.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rec8 -o rec8 -- python3 scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 --exchange records --no-pipeline --out gpurun_out/loop8_records_prof.json > gpurun_out/prof_rec8.log 2>&1
echo "exit $?"
