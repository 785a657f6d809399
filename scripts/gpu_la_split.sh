# Split look-ahead (OI_LA_SPLIT): GPU parity tests, per-launch timeline, eighth-day A/B, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u scripts/launch_perf2.py > gpurun_out/launch2.log 2>&1 || { tail -30 gpurun_out/launch2.log; exit 1; }
grep -E "k_chol_panel|k_diag_factor|totals" gpurun_out/launch2.log | grep -E "j= *(1|7|25|43|45)|totals"
for v in 1 0 1 0; do
  OI_LA_SPLIT=$v timeout -k 10 300 python bench.py --workload dayshard --no-cpu-baseline --out gpurun_out/ab_$v.json > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));r=d['roofline'];print('split=$v', d['value'], {k: r['kernels_ms'][k] for k in ('k_chol_panel','k_diag_factor','k_panel_even')})"
done
timeout -k 10 900 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('bench', d['value'], r['kernel'], r['achieved'], r['frac'], r['frac_executed'], r['kernels_ms'], d['cpu_baseline']['value'])"
