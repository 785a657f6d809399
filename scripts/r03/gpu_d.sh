#!/bin/bash
# round 3: k_panel4 (two block rows per workgroup, 128x128 core) -- parity,
# per-kernel A/B at fixed sizes, the day with OI_PANEL4=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03d
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "panel4 or alternate or schemes" > $D/gputests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $D/gputests.log | tail -12; [ $rc -eq 0 ] || exit $rc
for p in 0 1; do
  OI_PANEL4=$p timeout -k 10 300 python3 scripts/quick_perf.py > $D/quick_perf_p4_$p.txt 2>&1 || exit 1
  echo "== OI_PANEL4=$p"; grep -E "SMLII|panel|chol" $D/quick_perf_p4_$p.txt
done
OI_PANEL4=1 timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day_p4.json 2> $D/bench_day_p4.err || { tail -20 $D/bench_day_p4.err; exit 1; }
grep "GPU leg" $D/bench_day_p4.err; python3 -c "import json;d=json.load(open('$D/bench_day_p4.json'));r=d['roofline'];print(r['frac'],r['kernels_ms'],r['gemm_kernels'], d['parity'])"
