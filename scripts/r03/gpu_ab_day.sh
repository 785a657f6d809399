#!/bin/bash
# round 3: back-to-back day runs of the in-tree library and an A/B variant (OI_LIB=$1), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03abday
mkdir -p $D
for rep in 1 2; do
  for v in cur alt; do
    if [ $v = alt ]; then export OI_LIB=$1; else unset OI_LIB; fi
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline > $D/day_${v}_$rep.json 2> $D/day_${v}_$rep.err || { tail -5 $D/day_${v}_$rep.err; exit 1; }
    echo "$v $rep $(grep 'GPU leg' $D/day_${v}_$rep.err)"
  done
done
