# round 5, first call: the self-launch test and the 2-rank bitwise test, then
# the driver's exact bench command on the round-5 tree (baseline)
set -o pipefail
D=gpurun_out/r05/a; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $D/multirank.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" $D/multirank.log | tail -5; [ $rc -eq 0 ] || { tail -60 $D/multirank.log; exit $rc; }
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $D/bench_day.json > $D/bench_day.log 2>&1 || { tail -20 $D/bench_day.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_day.json')); c=d['cpu_baseline']; r=d['roofline']
print('day', d['value'], r['kernel'], r['frac'], {k: v['ms'] for k, v in r['gemm_kernels'].items()}, r['kernels_ms'].get('k_build'), 'cpu', c['value'], d['parity']['pass'], d['ranks_seen'], d['launcher'])"
