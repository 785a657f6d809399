#!/bin/bash
# Round-4 GPU steps in one parameterised driver (replaces the thirteen one-off
# scripts/gpu_r04_[a-m].sh; the outputs they wrote are under profiles/r04/).
# Usage: bash scripts/r04/run.sh STEP [STEP ...]   (every step has its own
# time limit; the first failing step ends the call)
#   eigh-probe      tools/eigh_probe 928 32 (phase times of oila::eigh)
#   eigh-trace      rocprofv3 kernel trace + stats of the probe
#   gemm4-probe     tools/gemm4_probe (LDS-DMA / 256x128 core variants)
#   nystrom-tests   tests/test_gpu_nystrom.py
#   nystrom-bench   bench.py --workload nystrom --steps ${STEPS:-10}
#   shares          the 8 config-4 shares of the day back to back (scripts/r04/gpu_shares.sh, DEPTH)
#   gpu-tests       the whole -m gpu suite
#   day             the driver's bench command (cpu_baseline from the day fixture)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r04/run; mkdir -p $D
for step in "$@"; do
  case $step in
    eigh-probe) timeout -k 10 120 tools/eigh_probe 928 32 > $D/eigh_probe.txt 2>&1 && cat $D/eigh_probe.txt ;;
    eigh-trace) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- tools/eigh_probe 928 32 > $D/probe.txt 2>&1 &&
                find $D/t -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \; ;;
    gemm4-probe) timeout -k 10 120 ./tools/gemm4_probe > $D/g4probe.txt 2>&1 && cat $D/g4probe.txt ;;
    nystrom-tests) timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/nys_tests.log 2>&1; rc=$?; tail -2 $D/nys_tests.log; [ $rc -eq 0 ] ;;
    nystrom-bench) timeout -k 10 600 python3 bench.py --workload nystrom --steps ${STEPS:-10} --warmup 2 --out $D/bench_nystrom.json > $D/bench_nystrom.log 2>&1 &&
                   python3 -c "import json; d=json.load(open('$D/bench_nystrom.json')); print('nystrom', d['value'], d['roofline']['stages_ms'])" ;;
    shares) bash scripts/r04/gpu_shares.sh > $D/shares.txt 2>&1; rc=$?; tail -30 $D/shares.txt; [ $rc -eq 0 ] ;;
    gpu-tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gputests.log 2>&1; rc=$?; grep -E "passed|failed" $D/gputests.log | tail -2; [ $rc -eq 0 ] ;;
    day) timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $D/bench_day.json > $D/bench_day.log 2>&1 &&
         python3 -c "import json; d=json.load(open('$D/bench_day.json')); print('day', d['value'], d['roofline']['kernel'], d['roofline']['frac'])" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac || { echo "step $step failed"; exit 1; }
done
