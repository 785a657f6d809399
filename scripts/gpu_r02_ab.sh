#!/bin/bash
# A/B of engine knobs on the driver's bench command (no CPU baseline).
# Each variant is "ENV=V ENV2=V2;extra bench args" (either part may be empty).
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
i=0
for v in "$@"; do
  i=$((i+1))
  envs="${v%%;*}"; args="${v#*;}"
  env $envs timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $args > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err
  rc=$?; echo "[$v] rc $rc $(grep 'GPU leg' gpurun_out/ab_${TAG}_$i.err)"
  [ $rc -eq 0 ] || exit $rc
done
