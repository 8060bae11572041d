#!/bin/bash
# One gpurun call = a list of named steps, each under its own time limit; output under
# gpurun_out/<tag>/. Stops at the first failing step (never retries a GPU step).
#   gpurun -- 'bash scripts/gpu_steps.sh r2x tests bench cfg4 prof_cfg4'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export PYTHONPATH=$PWD
test -f mxstream/_mxs_native*.so || { echo "native module missing"; exit 3; }
prof() {  # prof <name> <cmd...>: rocprofv3 kernel trace + stats of one python command
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_$name" -o "$name" -- "$@" \
     > "$out/prof_$name.log" 2>&1)
}
for step in "$@"; do
  echo "== $step"
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
           st=$?; tail -3 "$out/pytest_gpu.log"; [ $st -eq 0 ] || [ $st -eq 1 ] || exit $st ;;
    t_*) f=${step#t_}; timeout -k 10 600 python -u -m pytest tests/test_$f.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$out/pytest_$f.log" 2>&1
         st=$?; tail -3 "$out/pytest_$f.log"; [ $st -eq 0 ] || exit $st ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $? ;;
    bench) timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench.log" 2>&1 || exit $? ;;
    bench_nopipe) timeout -k 10 300 python bench.py --steps 48 --warmup 8 --no-pipeline > "$out/bench_nopipe.log" 2>&1 || exit $? ;;
    bench_hashed) timeout -k 10 300 python bench.py --steps 48 --warmup 8 --hashed-keys > "$out/bench_hashed.log" 2>&1 || exit $? ;;
    prof_bench_hashed) prof bench_hashed python3 bench.py --steps 24 --warmup 6 --hashed-keys || exit $? ;;
    bench_sync_*) m=${step#bench_sync_}; MXS_SYNC=$m timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench_sync_$m.log" 2>&1 || exit $? ;;
    bench_times) MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench_times.log" 2>&1 || exit $? ;;
    bench_sprof*) MXS_STEP_TIMES=1 MXS_STEP_PROFILE=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/$step.log" 2>&1 || exit $? ;;
    bench_k32) MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 --int32-keys > "$out/bench_k32.log" 2>&1 || exit $? ;;
    prof_k32) prof k32 python3 bench.py --steps 24 --warmup 6 --int32-keys || exit $? ;;
    bench_nopair) MXS_PAIR=0 MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench_nopair.log" 2>&1 || exit $? ;;
    bench_k32_nopair) MXS_PAIR=0 MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 --int32-keys > "$out/bench_k32_nopair.log" 2>&1 || exit $? ;;
    prof_nopair) MXS_PAIR=0 prof nopair python3 bench.py --steps 24 --warmup 6 || exit $? ;;
    bench_nofast) MXS_PART_FAST=0 MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench_nofast.log" 2>&1 || exit $? ;;
    prof_nofast) MXS_PART_FAST=0 prof nofast python3 bench.py --steps 24 --warmup 6 || exit $? ;;
    bench_nofin) MXS_FUSED_FIN=0 MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 > "$out/bench_nofin.log" 2>&1 || exit $? ;;
    prof_nofin) MXS_FUSED_FIN=0 prof nofin python3 bench.py --steps 24 --warmup 6 || exit $? ;;
    bench_zipf_*) z=${step#bench_zipf_}; MXS_STEP_TIMES=1 timeout -k 10 300 python bench.py --steps 48 --warmup 8 --zipf "$z" > "$out/bench_zipf_$z.log" 2>&1 || exit $? ;;
    prof_zipf_*) z=${step#prof_zipf_}; prof "zipf_$z" python3 bench.py --steps 24 --warmup 6 --zipf "$z" || exit $? ;;
    cfg6z_*) z=${step#cfg6z_}; z=${z%_*}; m=${step##*_}; extra=""; [ "$m" = valu ] && extra=--valu; timeout -k 10 300 python -m mxstream.models.bench_configs --config 6 --steps 20 --warmup 5 --zipf "$z" $extra > "$out/$step.json" 2>&1 || exit $? ;;
    cfg5r) timeout -k 10 300 python -m mxstream.models.bench_configs --config 5 --steps 20 --warmup 14 --revisit 0.01 > "$out/cfg5r.json" 2>&1 || exit $? ;;
    bench20) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$out/bench20.log" 2>&1 || exit $? ;;
    cfg1) timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --steps 20 --warmup 3 > "$out/cfg1.json" 2>&1 || exit $? ;;
    cfg1t*) t=${step#cfg1t}; timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --threads $t --steps 20 --warmup 3 > "$out/cfg1_t$t.json" 2>&1 || exit $? ;;
    cfg1gpu) timeout -k 10 300 python -m mxstream.models.bench_configs --config 1 --gpu-parse --steps 20 --warmup 3 > "$out/cfg1_gpu.json" 2>&1 || exit $? ;;
    cfg4_hashed) timeout -k 10 300 python -m mxstream.models.bench_configs --config 4 --hashed-keys --steps 20 --warmup 5 > "$out/cfg4_hashed.json" 2>&1 || exit $? ;;
    cfg7) timeout -k 10 600 python -m mxstream.models.bench_configs --config 7 > "$out/cfg7.json" 2>&1 || exit $? ;;
    cfg8) timeout -k 10 300 python -m mxstream.models.bench_configs --config 8 --steps 24 --warmup 13 > "$out/cfg8.json" 2>&1 || exit $? ;;
    cfg2|cfg4|cfg5|cfg6) timeout -k 10 300 python -m mxstream.models.bench_configs --config ${step#cfg} --steps 20 --warmup 5 > "$out/$step.json" 2>&1 || exit $? ;;
    loop8) timeout -k 10 300 python scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 --out "$out/loop8.json" > "$out/loop8.log" 2>&1 || exit $? ;;
    prof_bench) prof bench python3 bench.py --steps 24 --warmup 6 || exit $? ;;
    prof_bench_cap*) c=${step#prof_bench_cap}; prof bench_cap$c python3 bench.py --steps 24 --warmup 6 --cap-log2 $c || exit $? ;;
    pmc_bench*) # pmc_bench<k>: one counter pass over the headline (window_agg / partition)
      k=${step#pmc_bench}
      case $k in
        1) set="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" ;;
        2) set="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY" ;;
        3) set="TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum" ;;
      esac
      (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
       timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $set -d "$out/pmc_bench$k" -o run -- python3 bench.py --steps 6 --warmup 3 > "$out/pmc_bench$k.log" 2>&1) || exit $? ;;
    prof_cfg2|prof_cfg4|prof_cfg5|prof_cfg6) c=${step#prof_cfg}; prof cfg$c python3 -m mxstream.models.bench_configs --config $c --steps 12 --warmup 4 || exit $? ;;
    prof_loop8) prof loop8 python3 scripts/loopback_bench.py --world 8 --steps 24 --warmup 4 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
