# rocprofv3 kernel stats + the two PMC traffic passes over the default bench
# (the whole day on one GPU), no priming call so every dispatch is a timed one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmcd_fetch gpurun_out/pmcd_write
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-prime --out gpurun_out/bench_prof.json > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
grep -E "panel_even" gpurun_out/prof/run_kernel_stats.csv
timeout -s KILL 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcd_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --no-prime --out gpurun_out/bench_pmcd_fetch.json > gpurun_out/pmcd_fetch.log 2>&1 || { tail -30 gpurun_out/pmcd_fetch.log; exit 1; }
timeout -s KILL 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcd_write -o run --output-format csv -- python bench.py --no-cpu-baseline --no-prime --out gpurun_out/bench_pmcd_write.json > gpurun_out/pmcd_write.log 2>&1 || { tail -30 gpurun_out/pmcd_write.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmcd_fetch gpurun_out/pmcd_write > gpurun_out/pmcd_summary.json
python -c "
import json; d=json.load(open('gpurun_out/pmcd_summary.json'))['kernels']
for k in ('k_panel_even','k_chol_panel','k_lauum_grad1'):
    v=d.get(k); print(k, v and (v['dispatches'], round(v['hbm_bytes_per_dispatch']/1e9,3), 'GB/launch'))
"
