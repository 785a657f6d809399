#!/bin/bash
# session pipeline depth / resident-cell pool on the final tree (submit stream): the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/depth
mkdir -p $D
for cfg in "8 4096" "19 4096" "8 6144" "19 6144"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --depth $1 --max-pool $2 > $D/day_d$1_p$2.json 2> $D/day_d$1_p$2.err || exit 1
  echo "depth $1 pool $2"; grep "GPU leg" $D/day_d$1_p$2.err
done
