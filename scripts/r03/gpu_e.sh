#!/bin/bash
# round 3: day A/B (k_panel_even vs k_panel4, back to back on one box), then the
# config-5 share (12.5 km season day, 1/8 of its cells, n up to 5000)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03e
mkdir -p $D
for p in 1 0; do
  OI_PANEL4=$p timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline > $D/bench_day_p4_$p.json 2> $D/bench_day_p4_$p.err || { tail -20 $D/bench_day_p4_$p.err; exit 1; }
  echo "OI_PANEL4=$p $(grep 'GPU leg' $D/bench_day_p4_$p.err)"
done
timeout -k 10 1050 python3 bench.py --workload season --gpus 1 --steps 20 --warmup 5 --budget-s 1000 --dump $D/season_cells.npz > $D/bench_season.json 2> $D/bench_season.err || { tail -20 $D/bench_season.err; exit 1; }
grep "GPU leg" $D/bench_season.err; python3 -c "import json;d=json.load(open('$D/bench_season.json'));print(d['value'],d['evals_per_cell'],d['roofline']['frac'],d.get('parity'),d['cpu_baseline'].get('value'), d.get('truncated'))"
