# full GPU suite under OI_PANEL=2, then default-bench A/B (warmup 1, steps 2) of both schemes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OI_PANEL=2 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_p2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_p2.log; exit 1; }
echo "OI_PANEL=2 suite: $(tail -n 1 gpurun_out/gpu_tests_p2.log)"
for v in 2 1 2 1; do
  OI_PANEL=$v timeout -k 10 600 python bench.py --no-cpu-baseline --out gpurun_out/bench_p.json > gpurun_out/bench_p.log 2>&1 || { tail -30 gpurun_out/bench_p.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_p.json'))
r=d['roofline']; k=r['kernels_ms']; print('OI_PANEL=$v value', d['value'], 'evals', d['evals_per_cell'], 'dom', r['kernel'], r['achieved'], 'even', k['k_panel_even'], 'odd/legacy', k['k_chol_panel'], 'lauum', k['k_lauum_grad'], 'scale', k['k_scale'])"
done
