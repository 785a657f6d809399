# round 4: the 1-GPU day line (driver command, cpu_baseline from the day
# fixture) and config 4's 8 shares at depth 8 and 20 on the same box
set -o pipefail
D=gpurun_out/r04/day; mkdir -p $D
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $D/bench_day.json > $D/bench_day.log 2>&1 || { tail -20 $D/bench_day.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_day.json')); c=d['cpu_baseline']
print('day', d['value'], d['roofline']['kernel'], d['roofline']['frac'], 'cpu', c['value'], {k: c.get(k) for k in ('e_cpu_mean_timed_cells','fit_time_residual_max_abs') if k in c})"
for dep in 8 20; do
  DEPTH=$dep timeout -k 10 500 bash scripts/r04/gpu_shares.sh > $D/shares_d$dep.txt 2>&1 || { tail -20 $D/shares_d$dep.txt; exit 1; }
  python3 scripts/r04/share_projection.py gpurun_out/r04/shares_d$dep $D/bench_day.json | grep -E "projected|max_share|one_gpu"
done
