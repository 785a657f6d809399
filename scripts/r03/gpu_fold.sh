#!/bin/bash
# round 3: folded pair step (k_diag_pair + k_panel_pair) -- parity first, then
# the per-kernel probe and the day without the CPU legs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03fold
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/parity.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $D/parity.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_session.py tests/test_gpu_fit.py tests/test_gpu_gpr_surface.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/more.log 2>&1
rc=$?; tail -3 $D/more.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/quick_perf.py > $D/quick_perf.txt 2>&1 && cat $D/quick_perf.txt || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err; python3 -c "import json;d=json.load(open('$D/bench_day.json'));r=d['roofline'];print(d['value'],d.get('parity'));print(r['frac'],r['kernels_ms'],r['gemm_kernels'])"
