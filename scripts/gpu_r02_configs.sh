#!/bin/bash
# round 2: GPU tests, the driver's bench command, config 2 (predict) and config 1 (single cell)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc $rc"; grep "GPU leg" gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --workload predict --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_predict.json 2> gpurun_out/bench_${TAG}_predict.err
rc=$?; echo "predict rc $rc"; grep "GPU leg" gpurun_out/bench_${TAG}_predict.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_single.json 2> gpurun_out/bench_${TAG}_single.err
rc=$?; echo "single rc $rc"; grep "GPU leg" gpurun_out/bench_${TAG}_single.err
exit $rc
