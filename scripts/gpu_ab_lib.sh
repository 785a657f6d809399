# A/B of library builds: $@ = list of .so names in optimalinterpolation_amd/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export OI_DEBUG=1
for so in "$@"; do
  OI_LIB=$PWD/optimalinterpolation_amd/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_par.log 2>&1 || { grep "oi debug" gpurun_out/ab_par.log; tail -30 gpurun_out/ab_par.log; exit 1; }
  echo "$so parity: $(tail -n 1 gpurun_out/ab_par.log)"; grep "oi debug" gpurun_out/ab_par.log | grep -v "n=2 " | head -3 || true
done
for rep in 1 2; do
for so in "$@"; do
  OI_LIB=$PWD/optimalinterpolation_amd/$so timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_ab.json > gpurun_out/bench_ab.log 2>&1 || { tail -30 gpurun_out/bench_ab.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_ab.json'))
r=d['roofline']; k=r['kernels_ms']; print('$so value', d['value'], 'panel', k['k_chol_panel'], 'lauum', k['k_lauum_grad'], 'scale', k['k_scale'], 'diag', k['k_diag_factor'])"
done
done
