#!/bin/bash
# rolled vs unrolled k_lauum_grad1 epilogue: parity tests, one-round probe, the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/rolled
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/parity.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $D/parity.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $D/parity.log | head; exit $rc; }
timeout -k 10 120 python3 scripts/lauum_probe.py > $D/probe_rolled.txt 2>&1 || exit 1
OI_LIB=build_exp/liboi_unrolled.so timeout -k 10 120 python3 scripts/lauum_probe.py > $D/probe_unrolled.txt 2>&1 || exit 1
echo rolled; cat $D/probe_rolled.txt; echo unrolled; cat $D/probe_unrolled.txt
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_rolled.json 2> $D/day_rolled.err || exit 1
grep "GPU leg" $D/day_rolled.err
OI_LIB=build_exp/liboi_unrolled.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_unrolled.json 2> $D/day_unrolled.err || exit 1
grep "GPU leg" $D/day_unrolled.err
