#!/bin/bash
# One parameterised GPU launcher (replaces the per-round gpu_r*.sh scripts).
#
#   gpurun --timeout 1200 -- bash scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Each STEP is "name|seconds|command". Steps run in order, each under its own
# `timeout -k 10 seconds`, output in gpurun_out/TAG_name.log; the first failing step ends the
# run (a fault, abort or time limit leaves the GPU alone after it). The last line of each log
# is echoed so the gpurun tail carries the results. A command that starts with "prof:" runs
# under `rocprofv3 --kernel-trace --stats` from /tmp, output in gpurun_out/TAG_name/ ("pmem:"
# adds --memory-copy-trace).
#
# Shortcuts for STEP: "tests" (all GPU tests), "bench" (bench.py 24/6), "smoke" (__graft_entry__.smoke),
# "cfgN" (bench_configs --config N, default steps), "profN" (kernel profile of config N).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
export PYTHONPATH=$ROOT
mkdir -p gpurun_out
TAG=${1:?tag}
shift
expand() {
  if [[ $1 == *"|"* ]]; then echo "$1"; return; fi
  case "$1" in
    tests) echo "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" ;;
    bench) echo "bench|300|python bench.py --steps 24 --warmup 6" ;;
    smoke) echo "smoke|200|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" ;;
    cfg[0-9]*) echo "${1}|400|python -m mxstream.models.bench_configs --config ${1#cfg}" ;;
    prof[0-9]*) echo "${1}|400|prof:python3 -m mxstream.models.bench_configs --config ${1#prof} --steps 10 --warmup 6" ;;
    *) echo "$1" ;;
  esac
}
for raw in "$@"; do
  step=$(expand "$raw")
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  log="$ROOT/gpurun_out/${TAG}_${name}.log"
  t0=$(date +%s)
  if [[ $cmd == prof:* || $cmd == pmem:* ]]; then
    trace="--kernel-trace --stats"
    [[ $cmd == pmem:* ]] && trace="--kernel-trace --memory-copy-trace --stats"
    cmd=${cmd#prof:}
    cmd=${cmd#pmem:}
    (cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 "$secs" rocprofv3 $trace -d "$ROOT/gpurun_out/${TAG}_${name}" \
        -o prof -- $cmd > "$log" 2>&1)
  else
    timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  fi
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s :: $(tail -1 "$log" | cut -c1-600)"
  if [ $rc -ne 0 ]; then
    tail -25 "$log"
    exit $rc
  fi
done
echo "all steps ok"
