#!/bin/bash
# GPU parity suite + config 2 / config 1 / the day (no CPU baseline) on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/${1:-check2}
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" $D/gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $D/gputests.log | head -20; exit $rc; }
timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline > $D/predict.json 2> $D/predict.err || exit 1
grep "GPU leg" $D/predict.err
timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > $D/single.json 2> $D/single.err || exit 1
grep "GPU leg" $D/single.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day.json 2> $D/day.err || exit 1
grep "GPU leg" $D/day.err
