#!/bin/bash
# Round-6 GPU steps in one parameterised driver (round 5's scripts/r05/run.sh
# plus this round's steps; outputs under gpurun_out/r06/$TAG, copied to
# profiles/r06/ by hand).
# Usage: bash scripts/r06/run.sh STEP [STEP ...]   (every step has its own
# time limit; the first failing step ends the call)
#   gpu-tests       the -m gpu suite without the long T3 fits (FULL=1: all of it)
#   multirank       tests/test_gpu_multirank.py (self-launched ranks, 2-rank bitwise)
#   day             the driver's bench command (cpu_baseline from the day fixture)
#   day-ab          the day back to back against $OI_LIB_BASE (new base new base)
#   day-ab-env      the same against the knob setting $AB_ENV (e.g. AB_ENV=OI_LAUUM=4)
#   parity-env      the GPU parity / fit / session tests under $AB_ENV
#   shares          config 4's 8 day shares back to back on one GPU + projection (ONE_GPU_JSON)
#   day-8rank       8 self-launched gloo ranks sharing one GPU (OI_DIST_BACKEND=gloo)
#   config1         --workload single (one n = 200 cell, GPR:166)
#   config2         --workload predict (1000 cells x n = 500, GPR:316-319)
#   season          --workload season --season-days ${DAYS:-1} (config 5, one share)
#   nystrom-tests   tests/test_gpu_nystrom.py
#   nystrom-bench   bench.py --workload nystrom --steps ${STEPS:-10}
#   svgp-bench      bench.py --workload svgp
#   eigh-probe      tools/eigh_probe 928 64 (phase times and accuracy of oila::eigh)
#   gemm-probe      tools/gemm_probe 4600 928 32 for OI_GEMM128 = 1, 0
#   eigh-trace      rocprofv3 kernel trace + stats of the eigensolver probe
# round 6:
#   t1              tests/test_gpu_day_t1.py (GPU objective vs the reference's order noise), arrays dumped
#   t3              tests/test_gpu_day_fits.py + test_gpu_fit_large.py (T3), fits dumped
#   twopass         bench.py --workload twopass (the whole two-pass day, GPR:223-336)
#   cpu-model       scripts/r06/cpu_model_check.py (host only: the CPU-baseline model at n = 1500..3000)
#   pmc-tcc         TCC hit / miss / fabric-read counters of the day's kernels ($OI_LIB if set)
#   day-abn         the day over the builds in $LIBS ("cur" = the tree), round robin, $REPS rounds
#   config1-trace   rocprofv3 kernel trace of config 1: per-kernel durations and the gaps between launches
# Profiles of the driver's command: scripts/r05/gpu_prof.sh; end-of-round
# verification: scripts/r05/gpu_verify.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r06/${TAG:-run}; mkdir -p $D
show() {  # one summary line of a bench JSON
  python3 -c "
import json, sys; d = json.load(open(sys.argv[1])); r = d.get('roofline') or {}
print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], r.get('kernel'), r.get('frac'),
      (d.get('parity') or {}).get('pass'), d.get('ranks_seen'))" "$1" "$2"
}
bench() {  # bench LIMIT NAME ARGS...: one bench.py run into $D/NAME.json
  local lim=$1 name=$2; shift 2
  timeout -k 10 $lim python3 bench.py "$@" --out $D/$name.json > $D/$name.log 2>&1 || { tail -20 $D/$name.log; return 1; }
  show $D/$name.json $name
}
for step in "$@"; do
  case $step in
    gpu-tests)
      K="not fit_large and not day_fits"; [ "${FULL:-0}" = 1 ] && K=""
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${K:+-k "$K"} > $D/gputests.log 2>&1
      rc=$?; grep -E "passed|failed" $D/gputests.log | tail -2; [ $rc -eq 0 ] || grep -E "FAILED|Error" $D/gputests.log | head ;;
    multirank)
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $D/multirank.log 2>&1
      rc=$?; grep -E "passed|failed" $D/multirank.log | tail -2; [ $rc -eq 0 ] ;;
    day) bench 560 day --gpus 1 --steps 20 --warmup 5 ;;
    day-ab|day-ab-env)  # the day back to back: the build at $OI_LIB_BASE (day-ab) or the knob setting $AB_ENV
      # (day-ab-env, e.g. AB_ENV=OI_LAUUM=4) against the tree's default
      fail=0; k=0
      for leg in new base new base; do
        k=$((k + 1)); E=""
        if [ $step = day-ab ]; then [ $leg = base ] && E="OI_LIB=$OI_LIB_BASE"; else [ $leg = base ] && E="$AB_ENV"; fi
        [ $leg = base ] && [ -z "$OI_LIB_BASE$AB_ENV" ] && { echo "$step needs OI_LIB_BASE / AB_ENV"; fail=1; break; }
        env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 8 \
          --out $D/day_${leg}_$k.json > $D/day_${leg}_$k.log 2>&1 || { tail -20 $D/day_${leg}_$k.log; fail=1; break; }
        show $D/day_${leg}_$k.json "$leg($E)"
      done; [ $fail = 0 ] ;;
    parity-env)  # the GPU parity / fit tests under $AB_ENV
      env $AB_ENV timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py tests/test_gpu_session.py -x -q \
        --timeout 300 --timeout-method thread > $D/parity_env.log 2>&1
      rc=$?; tail -1 $D/parity_env.log; [ $rc -eq 0 ] || tail -30 $D/parity_env.log; [ $rc -eq 0 ] ;;
    shares)  # config 4 rehearsed on one GPU: the 8 LPT shares of the day back to back (the N = 8 depth rule),
      # then the projection (slowest share) against the 1-GPU line $ONE_GPU_JSON
      fail=0
      for k in 0 1 2 3 4 5 6 7; do
        bench 300 share_$k --gpus 1 --steps 20 --warmup 2 --day-shares 8 --share $k --no-cpu-baseline --parity-cells 0 || { fail=1; break; }
      done
      [ $fail = 0 ] && mkdir -p $D/shares && cp $D/share_*.json $D/shares/ &&
      python3 scripts/r04/share_projection.py $D/shares ${ONE_GPU_JSON:-} ;;
    day-8rank) OI_DIST_BACKEND=gloo bench 400 day_8rank_gloo --gpus 8 --steps 20 --warmup 2 --no-cpu-baseline --parity-cells 8 ;;
    config1) bench 300 config1 --workload single --steps 20 --warmup 3 ;;
    config2) bench 300 config2 --workload predict --steps 20 --warmup 3 ;;
    season) bench 1150 season --workload season --season-days ${DAYS:-1} --steps 21 --warmup 2 --budget-s 1000 --no-cpu-baseline --parity-cells 8 ;;
    nystrom-tests)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/nys_tests.log 2>&1
      rc=$?; tail -1 $D/nys_tests.log; [ $rc -eq 0 ] ;;
    nystrom-bench) bench 600 nystrom --workload nystrom --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ;;
    svgp-bench) bench 300 svgp --workload svgp --steps 1 --warmup 1 --no-cpu-baseline ;;
    eigh-probe) timeout -k 10 180 tools/eigh_probe 928 64 > $D/eigh_probe.txt 2>&1 && cat $D/eigh_probe.txt ;;
    gemm-probe)
      for g in 1 0; do OI_GEMM128=$g timeout -k 10 60 tools/gemm_probe 4600 928 32 | sed "s/^/gemm128=$g /" || exit 1; done | tee $D/gemm_probe.txt ;;
    eigh-trace)
      timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- tools/eigh_probe 928 64 > $D/probe.txt 2>&1 &&
      find $D/t -name "*kernel_stats.csv" -exec cp {} $D/eigh_kernel_stats.csv \; && rm -rf $D/t ;;
    t1)
      OI_T1_DUMP=$D/t1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_day_t1.py -x -v -s --timeout 300 \
        --timeout-method thread > $D/t1.log 2>&1
      rc=$?; grep -E "d_gpu|passed|failed" $D/t1.log | tail -30; [ $rc -eq 0 ] ;;
    t3)
      OI_T3_DUMP=$D/t3 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_day_fits.py tests/test_gpu_fit_large.py -v -s \
        --timeout 600 --timeout-method thread > $D/t3.log 2>&1
      rc=$?; grep -E "OI_DEDUP|GPU|passed|failed" $D/t3.log | tail -40; [ $rc -eq 0 ] ;;
    twopass) bench 900 twopass --workload twopass --steps 1 --parity-cells ${PCELLS:-24} ;;
    cpu-model)
      timeout -k 10 1150 python3 -u scripts/r06/cpu_model_check.py --out $D/cpu_model_check.json > $D/cpu_model.log 2>&1
      rc=$?; tail -5 $D/cpu_model.log; [ $rc -eq 0 ] ;;
    pmc-tcc)
      CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline"
      timeout -s KILL 420 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $D/pmcT -o run \
        --output-format csv -- $CMD > $D/pmcT.json 2> $D/pmcT.err
      rc=$?; echo "tcc rc $rc"; [ $rc -eq 0 ] || { tail -5 $D/pmcT.err; exit $rc; }
      python3 scripts/pmc_kernels.py $D/pmcT > $D/pmc_tcc${OI_LIB:+_$(basename $OI_LIB .so)}.txt && rm -rf $D/pmcT
      cut -c1-260 $D/pmc_tcc*.txt | head -8 ;;
    day-abn)  # the day over the builds in $LIBS ("cur" = the tree's liboi.so), round robin, ${REPS:-2} rounds
      fail=0; k=0
      for rep in $(seq ${REPS:-2}); do for lib in $LIBS; do
        k=$((k + 1)); E=""; [ $lib != cur ] && E="OI_LIB=$lib"; tag=$(basename $lib .so)
        env $E timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 8 \
          --out $D/day_${tag}_$k.json > $D/day_${tag}_$k.log 2>&1 || { tail -20 $D/day_${tag}_$k.log; fail=1; break 2; }
        show $D/day_${tag}_$k.json "$tag"
        python3 -c "import json,sys; r=json.load(open(sys.argv[1]))['roofline']; print('   ', {k: round(v / 1e3, 3) for k, v in r['kernels_ms'].items() if v > 100})" $D/day_${tag}_$k.json
      done; done; [ $fail = 0 ] ;;
    config1-trace)  # kernel durations and inter-kernel gaps of config 1 (one n = 200 cell per step)
      timeout -k 10 300 rocprofv3 --kernel-trace -d $D/c1t -o run --output-format csv -- python3 bench.py --workload single \
        --steps 10 --warmup 2 --no-cpu-baseline --timed-profile off > $D/config1_trace.json 2> $D/config1_trace.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 $D/config1_trace.err; exit $rc; }
      python3 scripts/trace_summary.py $D/c1t > $D/config1_trace_summary.txt && rm -rf $D/c1t && cat $D/config1_trace_summary.txt ;;
    *) echo "unknown step $step"; false ;;
  esac || { echo "step $step failed"; exit 1; }
done
