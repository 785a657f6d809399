#!/bin/bash
# GPU test suite, then an A/B of engine knobs on the driver's bench command
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/gputests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r02_ab.sh $TAG "$@"
