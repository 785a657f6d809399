# parity (all GPU tests) then A/B of the panel schemes on one bench step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/gpu_tests.log
for v in 0 1; do
OI_PANEL=$v timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_p$v.json > gpurun_out/bench_p.log 2>&1 || { tail -30 gpurun_out/bench_p.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_p$v.json'))
r=d['roofline']; print('OI_PANEL=$v value', d['value'], 'evals', d['evals_per_cell'], 'dom', r['kernel'], r['achieved'], r['kernels_ms'])"
done
