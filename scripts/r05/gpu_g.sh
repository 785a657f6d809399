# round 5: config 5 on one GPU over three consecutive season days (seeds
# 0, 1, 2): each day's 1/8 share (~5000 cells, n ~ U{300..5000}) through one
# session, days in order; parity block of the timed cells
set -o pipefail
D=gpurun_out/r05/g; mkdir -p $D
timeout -k 10 1150 python3 bench.py --workload season --season-days 3 --steps 21 --warmup 2 --budget-s 1000 --no-cpu-baseline --parity-cells 8 --out $D/season_3days.json > $D/season_3days.log 2>&1 || { tail -20 $D/season_3days.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/season_3days.json')); r=d['roofline']
print('season 3 days', d['value'], d['timed_s'], d.get('truncated'), d['config']['cells_total'], d['evals_per_cell'], r['kernel'], r['frac'], d['parity'])"
