#!/bin/bash
# round-2 final numbers: the driver's exact command (CPU baseline included), config 1, config 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_day.json 2> gpurun_out/bench_${TAG}_day.err
rc=$?; echo "day rc $rc"; grep "GPU leg" gpurun_out/bench_${TAG}_day.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_single.json 2> gpurun_out/bench_${TAG}_single.err || exit 1
grep "GPU leg" gpurun_out/bench_${TAG}_single.err
timeout -k 10 300 python3 bench.py --workload predict --steps 50 --warmup 5 > gpurun_out/bench_${TAG}_predict.json 2> gpurun_out/bench_${TAG}_predict.err || exit 1
grep "GPU leg" gpurun_out/bench_${TAG}_predict.err
timeout -k 10 200 python3 scripts/single_latency.py 200 8 > gpurun_out/single_${TAG}.json 2> gpurun_out/single_${TAG}.err || exit 1
grep -A2 '"profile=False"' gpurun_out/single_${TAG}.json
