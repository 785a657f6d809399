#!/bin/bash
# Round-5 GPU steps in one parameterised driver (replaces the one-off
# scripts/r05/gpu_[a-z].sh of this round; the outputs they wrote are under
# profiles/r05/, the per-experiment directory named in DESIGN §4c / §6.0).
# Usage: bash scripts/r05/run.sh STEP [STEP ...]   (every step has its own
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
# Profiles of the driver's command: scripts/r05/gpu_prof.sh; end-of-round
# verification: scripts/r05/gpu_verify.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r05/${TAG:-run}; mkdir -p $D
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
    *) echo "unknown step $step"; false ;;
  esac || { echo "step $step failed"; exit 1; }
done
