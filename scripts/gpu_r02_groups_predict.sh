#!/bin/bash
# config 2 with 1 / 2 / 3 resident-cell stream groups (submit stream no longer drains the groups)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/gp
mkdir -p $D
for g in 1 2 3 1 2 3; do
  OI_GROUPS=$g timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline > $D/predict_g$g.json 2> $D/predict_g$g.err || exit 1
  echo "groups $g"; grep "GPU leg" $D/predict_g$g.err
done
for g in 1 2; do
  OI_GROUPS=$g timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline --max-pool 8192 --depth 16 > $D/predict_big_g$g.json 2> $D/predict_big_g$g.err || exit 1
  echo "pool 8192 depth 16 groups $g"; grep "GPU leg" $D/predict_big_g$g.err
done
