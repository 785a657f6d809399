# one GPU iteration: parity tests, SMLII batch perf, short bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
timeout -k 10 300 python scripts/quick_perf.py > gpurun_out/perf.log 2>&1 || { tail -30 gpurun_out/perf.log; exit 1; }
cat gpurun_out/perf.log
timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_iter.json > gpurun_out/bench_iter.log 2>&1 || { tail -30 gpurun_out/bench_iter.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_iter.json'))
r=d['roofline']; print('value', d['value'], 'cells/s; evals/cell', d['evals_per_cell'], '; useful TF', r['useful_tflops_per_gpu'], '; dom', r['kernel'], r['achieved'], 'TF'); print(r['kernels_ms'])"
