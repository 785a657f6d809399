# HBM traffic per kernel launch of the default bench step: two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE), kernel trace only; summary -> gpurun_out/pmc_summary.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prime --out gpurun_out/bench_pmc_fetch.json > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prime --out gpurun_out/bench_pmc_write.json > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.json && python -c "import json;d=json.load(open('gpurun_out/pmc_summary.json'));print({k:v['hbm_bytes_per_launch'] for k,v in d.items() if k.startswith('k_')})"
