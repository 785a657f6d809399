# Full round check: all GPU tests, smoke, default bench (the whole day on one
# GPU), rocprofv3 kernel stats of the same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -n 3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-prime --out gpurun_out/bench_prof.json > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \;
