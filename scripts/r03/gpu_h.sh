#!/bin/bash
# round 3: where k_panel4 pays -- even column threshold sweep (fixed sizes), then the day at two settings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03h
mkdir -p $D
for mj in 0 4 8 12 1000; do
  OI_PANEL4_MINJ=$mj timeout -k 10 200 python3 scripts/quick_perf.py > $D/quick_minj_$mj.txt 2>&1 || exit 1
  echo "minj=$mj $(grep -E 'config2|SMLII' $D/quick_minj_$mj.txt | tr '\n' ' ' | cut -c1-400)"
done
for mj in 8 0; do
  OI_PANEL4_MINJ=$mj timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline > $D/bench_day_minj_$mj.json 2> $D/bench_day_minj_$mj.err || exit 1
  echo "day minj=$mj $(grep 'GPU leg' $D/bench_day_minj_$mj.err)"
done
