#!/bin/bash
# GPU parity suite (k_build lower-triangle diagonal tiles, post-form, OI_RING=3 case), then
# the day and config 2 with the two- vs three-deep register ring in k_panel_even
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/ring
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" $D/gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $D/gputests.log | head -20; exit $rc; }
for r in 2 3 2 3; do
  OI_RING=$r timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline > $D/predict_r$r.json 2> $D/predict_r$r.err || exit 1
  echo "ring $r"; grep "GPU leg" $D/predict_r$r.err
done
timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > $D/single.json 2> $D/single.err || exit 1
grep "GPU leg" $D/single.err
for r in 2 3; do
  OI_RING=$r timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_r$r.json 2> $D/day_r$r.err || exit 1
  echo "ring $r"; grep "GPU leg" $D/day_r$r.err
done
