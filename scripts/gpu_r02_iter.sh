#!/bin/bash
# one iteration: diag probe, GPU tests, config-1 latency probe, config 2 and the day (driver command, no CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 60 ./tools/diag_engine_probe_rsq0 > gpurun_out/diagprobe0_$TAG.txt 2>&1 && grep -A0 engine gpurun_out/diagprobe0_$TAG.txt && timeout -k 10 60 ./tools/diag_engine_probe > gpurun_out/diagprobe_$TAG.txt 2>&1 || exit 1
grep engine gpurun_out/diagprobe_$TAG.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/single_latency.py 200 8 > gpurun_out/single_$TAG.json 2> gpurun_out/single_$TAG.err || exit 1
grep -A2 '"profile=False"' gpurun_out/single_$TAG.json
timeout -k 10 200 python3 bench.py --workload predict --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${TAG}_predict.json 2> gpurun_out/bench_${TAG}_predict.err || exit 1
grep -h "GPU leg" gpurun_out/bench_${TAG}_predict.err
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc $rc"; grep "GPU leg" gpurun_out/bench_$TAG.err
exit $rc
