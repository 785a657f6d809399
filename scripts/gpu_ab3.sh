# parity then A/B: panel scheme x lauum variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/gpu_tests.log
for cfg in "0 1" "1 1" "0 0" "1 0"; do
set -- $cfg
OI_PANEL=$1 OI_LAUUM=$2 timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_ab.json > gpurun_out/bench_ab.log 2>&1 || { tail -30 gpurun_out/bench_ab.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_ab.json'))
r=d['roofline']; k=r['kernels_ms']; print('PANEL=$1 LAUUM=$2 value', d['value'], 'panel_even', k['k_panel_even'], 'chol_panel', k['k_chol_panel'], 'lauum', k['k_lauum_grad'], 'scale', k['k_scale'])"
done
