# round 5: the one-workgroup round for small cells (k_eval_small) -- the GPU
# suite, config 1 (one n = 200 cell) and config 2 lines -- and the 8-rank
# self-launched day rehearsed on one GPU (gloo)
set -o pipefail
D=gpurun_out/r05/e1; mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fit_large and not day_fits" > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $D/gputests.log | tail -6; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $D/gputests.log | head -120; exit $rc; }
timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --out $D/config1.json > $D/config1.log 2>&1 || { tail -20 $D/config1.log; exit 1; }
OI_SMALL=0 timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline --out $D/config1_nosmall.json > $D/config1_nosmall.log 2>&1 || { tail -20 $D/config1_nosmall.log; exit 1; }
timeout -k 10 300 python3 bench.py --workload predict --steps 20 --warmup 3 --out $D/config2.json > $D/config2.log 2>&1 || { tail -20 $D/config2.log; exit 1; }
python3 -c "
import json
for f in ('config1', 'config1_nosmall', 'config2'):
    d = json.load(open('$D/' + f + '.json')); r = d['roofline']; c = d.get('cpu_baseline') or {}
    print(f, d['value'], d['ms_per_step'], r['kernel'], r['frac'], {k: round(v, 1) for k, v in r['kernels_ms'].items()}, c.get('value'))"
OI_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 8 --steps 20 --warmup 2 --no-cpu-baseline --parity-cells 8 --out $D/day_8rank_gloo.json > $D/day_8rank_gloo.log 2>&1 || { tail -30 $D/day_8rank_gloo.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/day_8rank_gloo.json')); print('8 ranks on 1 GPU', d['value'], d['n_gpus'], d['ranks_seen'], d['rank_devices'], d['collective_backend'], d['launcher'], d['config']['cells_total'], d['parity']['pass'])"
