set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_prof.json > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
ls -R gpurun_out/prof | head -20
cat gpurun_out/bench_prof.json
find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \;
