# bench lines of the other BASELINE configs: 2 (1000 x n=500 predict-only) and 1 (one cell, n=200)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload predict --steps 10 --warmup 2 --no-cpu-baseline --out gpurun_out/bench_config2.json > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
cat gpurun_out/bench_config2.json
timeout -k 10 300 python bench.py --workload single --steps 5 --warmup 1 --no-cpu-baseline --out gpurun_out/bench_config1.json > gpurun_out/bench_c1.log 2>&1 || { tail -20 gpurun_out/bench_c1.log; exit 1; }
cat gpurun_out/bench_config1.json
