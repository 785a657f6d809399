set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dayprof
timeout -k 10 600 python scripts/day_bench.py --out gpurun_out/day_bench.json > gpurun_out/day_bench.log 2>&1 || { tail -30 gpurun_out/day_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/day_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/dayprof -o run --output-format csv -- python scripts/day_bench.py --reps 1 --no-cpu > gpurun_out/dayprof.log 2>&1 || { tail -30 gpurun_out/dayprof.log; exit 1; }
find gpurun_out/dayprof -name "*kernel_stats.csv" -exec cat {} \;
