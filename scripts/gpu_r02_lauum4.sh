#!/bin/bash
# 64x64 (default) vs 128x128 (OI_LAUUM=4) K^-1 / gradient kernel on the final tree: the day, twice each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/lauum4
mkdir -p $D
for l in 1 4 1 4; do
  OI_LAUUM=$l timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/day_l$l.json 2> $D/day_l$l.err || exit 1
  echo "lauum $l"; grep "GPU leg" $D/day_l$l.err
  python3 -c "import json; d=json.load(open('$D/day_l$l.json')); print(d['roofline']['kernels_ms'])"
done
