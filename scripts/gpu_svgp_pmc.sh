# HBM traffic of the SVGP training launch: two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/svgp_fetch -o run --output-format csv -- python bench.py --workload svgp --no-cpu-baseline --no-prime --out gpurun_out/svgp_pmc_fetch.json > gpurun_out/svgp_pmc_fetch.log 2>&1 || { tail -20 gpurun_out/svgp_pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d /tmp/svgp_write -o run --output-format csv -- python bench.py --workload svgp --no-cpu-baseline --no-prime --out gpurun_out/svgp_pmc_write.json > gpurun_out/svgp_pmc_write.log 2>&1 || { tail -20 gpurun_out/svgp_pmc_write.log; exit 1; }
python scripts/pmc_summary.py /tmp/svgp_fetch /tmp/svgp_write > gpurun_out/svgp_pmc_summary.json
python -c "
import json; d=json.load(open('gpurun_out/svgp_pmc_summary.json'))['kernels']
print({k: (v['dispatches'], round(v['hbm_bytes_per_dispatch']/1e9,3)) for k, v in d.items()})"
