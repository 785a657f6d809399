#!/bin/bash
# config 1 (one n = 200 cell, --workload single) back to back: the tree's
# liboi.so against $OI_LIB_BASE, ${REPS:-2} rounds; outputs under $D
set -o pipefail
D=${D:?}; mkdir -p $D
for k in $(seq ${REPS:-2}); do
  for leg in base new; do
    E=""; [ $leg = base ] && E="OI_LIB=${OI_LIB_BASE:?}"
    env $E timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline \
      --out $D/c1_${leg}_$k.json > $D/c1_${leg}_$k.log 2>&1 || { tail -20 $D/c1_${leg}_$k.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'])" $D/c1_${leg}_$k.json $leg
  done
done
