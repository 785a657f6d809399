#!/bin/bash
# A/B of the diagonal-tile factor kernels: parity tests under the new default, then
# config 1 / config 2 / the day with OI_DIAG=16 (default) and OI_DIAG=32 (round 1)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02e}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
for v in 16 32; do
  OI_DIAG=$v timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_single_d$v.json 2> gpurun_out/bench_${TAG}_single_d$v.err || exit 1
  OI_DIAG=$v timeout -k 10 200 python3 bench.py --workload predict --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_predict_d$v.json 2> gpurun_out/bench_${TAG}_predict_d$v.err || exit 1
  grep -h "GPU leg" gpurun_out/bench_${TAG}_single_d$v.err gpurun_out/bench_${TAG}_predict_d$v.err
done
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc $rc"; grep "GPU leg" gpurun_out/bench_$TAG.err
exit $rc
