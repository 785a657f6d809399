# round 5: profiles of the driver's command on the round-5 tree (kernel trace +
# stats, FETCH_SIZE / WRITE_SIZE and SQ PMC passes; scripts/r05/gpu_prof.sh),
# then config 5's one-day share on this tree
set -o pipefail
SKIP_TESTS=1 bash scripts/r05/gpu_prof.sh r05 || exit $?
D=gpurun_out/r05/d; mkdir -p $D
timeout -k 10 560 python3 bench.py --workload season --steps 20 --warmup 2 --budget-s 520 --out $D/season_1day.json > $D/season_1day.log 2>&1 || { tail -20 $D/season_1day.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/season_1day.json')); r=d['roofline']
print('season', d['value'], d['timed_s'], r['kernel'], r['frac'], d['parity'], d['cpu_baseline']['value'])"
