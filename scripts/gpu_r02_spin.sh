#!/bin/bash
# polling (OI_SPIN=1, default) vs blocking round waits: config 1, config 2, the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/spin
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_session.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/tests.log 2>&1 || { tail -20 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for sp in 1 0 1 0; do
  OI_SPIN=$sp timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 --no-cpu-baseline > $D/single_s$sp.json 2> $D/single_s$sp.err || exit 1
  echo "spin $sp"; grep "GPU leg" $D/single_s$sp.err
done
for sp in 1 0; do
  OI_SPIN=$sp timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline > $D/predict_s$sp.json 2> $D/predict_s$sp.err || exit 1
  echo "spin $sp"; grep "GPU leg" $D/predict_s$sp.err
done
for sp in 1 0; do
  OI_SPIN=$sp timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_s$sp.json 2> $D/day_s$sp.err || exit 1
  echo "spin $sp"; grep "GPU leg" $D/day_s$sp.err
done
