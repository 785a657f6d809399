#!/bin/bash
# round 2: new GPU tests (session, multi-rank HIP path) + the driver's exact bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gputests_r02c.log 2>&1
echo "pytest rc $?"; tail -5 gpurun_out/gputests_r02c.log
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r02_day.json 2> gpurun_out/bench_r02_day.err
rc=$?; echo "bench rc $rc"; tail -3 gpurun_out/bench_r02_day.err; head -c 600 gpurun_out/bench_r02_day.json
exit $rc
