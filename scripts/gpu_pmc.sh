# HBM traffic of the bench step: two separate PMC passes (FETCH_SIZE, WRITE_SIZE),
# each with kernel trace only, plus the per-round timeline of one shard.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 python scripts/round_perf.py > gpurun_out/round.log 2>&1 || { tail -30 gpurun_out/round.log; exit 1; }
grep -v amdgpu.ids gpurun_out/round.log
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_pmc_fetch.json > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_pmc_write.json > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
ls -la gpurun_out/pmc_fetch gpurun_out/pmc_write
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.json && cat gpurun_out/pmc_summary.json
