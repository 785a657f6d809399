# round 4: g8 probe, Nystrom bench on the hand-written eigensolver, the driver's day command
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 ./tools/gemm4_probe > gpurun_out/r04/g8probe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 20 --warmup 2 --out gpurun_out/r04/bench_nystrom.json > gpurun_out/r04/bench_nystrom.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom.log; exit 1; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out gpurun_out/r04/bench_day.json > gpurun_out/r04/bench_day.log 2>&1 || { tail -20 gpurun_out/r04/bench_day.log; exit 1; }
cat gpurun_out/r04/g8probe.txt | tail -12
python3 - <<'PY'
import json
for f in ('bench_nystrom', 'bench_day'):
    d = json.load(open(f'gpurun_out/r04/{f}.json'))
    print(f, d['value'], d.get('evals_per_cell'), json.dumps(d.get('roofline', {}))[:400])
    print('  cpu', json.dumps(d.get('cpu_baseline'))[:600])
PY
