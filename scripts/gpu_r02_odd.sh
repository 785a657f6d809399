#!/bin/bash
# two-tile odd step (k_panel_odd, default) vs one-tile k_chol_panel (OI_ODD=1): GPU suite, day, configs 1/2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/odd
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" $D/gputests.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $D/gputests.log | head -20; exit $rc; }
for o in 2 1; do
  OI_ODD=$o timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_o$o.json 2> $D/day_o$o.err || exit 1
  echo "odd $o"; grep "GPU leg" $D/day_o$o.err
done
for o in 2 1; do
  OI_ODD=$o timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline > $D/predict_o$o.json 2> $D/predict_o$o.err || exit 1
  echo "odd $o"; grep "GPU leg" $D/predict_o$o.err
  OI_ODD=$o timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 --no-cpu-baseline > $D/single_o$o.json 2> $D/single_o$o.err || exit 1
  grep "GPU leg" $D/single_o$o.err
done
