# HBM traffic of the paired-panel scheme (OI_PANEL=2), same passes as gpu_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export OI_PANEL=2  # (now also the default)
mkdir -p gpurun_out/pmc2_fetch gpurun_out/pmc2_write
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc2_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_pmc2_fetch.json > gpurun_out/pmc2_fetch.log 2>&1 || { tail -30 gpurun_out/pmc2_fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc2_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_pmc2_write.json > gpurun_out/pmc2_write.log 2>&1 || { tail -30 gpurun_out/pmc2_write.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc2_fetch gpurun_out/pmc2_write > gpurun_out/pmc2_summary.json && python -c "
import json; d=json.load(open('gpurun_out/pmc2_summary.json'))['kernels']
for k in ('k_panel_even','k_chol_panel','k_lauum_grad1','k_scale'):
    v=d.get(k); print(k, v and (v['dispatches'], round(v['hbm_bytes_per_dispatch']/1e9,3), 'GB/launch'))
"
