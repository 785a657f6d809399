#!/bin/bash
# round 3: no column-(j+1) round trip at j = 0 -- parity, per-kernel times, the day with per-j totals
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03j0
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py -m gpu -x -q --timeout 200 --timeout-method thread > $D/parity.log 2>&1
rc=$?; tail -2 $D/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/r03/ab_probe.py j0skip > $D/ab.txt 2>&1 || exit 1
grep "\[" $D/ab.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline --dump $D/day.npz > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
