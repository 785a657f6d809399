#!/bin/bash
# round 2: full GPU test suite, the driver's exact bench command, and rocprofv3 of the same command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc $rc"; grep "GPU leg" gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
if [ "${2:-prof}" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_under_rocprof.json 2> gpurun_out/bench_${TAG}_under_rocprof.err
  rc=$?; echo "rocprof rc $rc"; find gpurun_out/prof_$TAG -name "*kernel_stats*" | head -3
fi
exit $rc
