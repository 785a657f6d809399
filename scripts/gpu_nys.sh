#!/bin/bash
# Nystrom variant: GPU parity tests, bench line, rocprof kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nystrom.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/nys_tests.log 2>&1 || { tail -40 gpurun_out/nys_tests.log; exit 1; }
grep -E "PASS|FAIL|rel|passed|failed" gpurun_out/nys_tests.log | tail -12
timeout -k 10 300 python bench.py --workload nystrom --steps 1 --warmup 0 ${NYS_BENCH_ARGS} --out gpurun_out/nys_bench.json > gpurun_out/nys_bench.log 2>&1 || { tail -30 gpurun_out/nys_bench.log; exit 1; }
cat gpurun_out/nys_bench.json
if [ -n "$NYS_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/nys_prof -o nys --output-format csv -- python bench.py --workload nystrom --steps 1 --warmup 0 --no-cpu-baseline --no-prime --out gpurun_out/nys_bench_prof.json > gpurun_out/nys_prof.log 2>&1 || { tail -30 gpurun_out/nys_prof.log; exit 1; }
f=$(find /tmp/nys_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/nys_kernel_stats.csv
head -14 gpurun_out/nys_kernel_stats.csv | cut -c1-180
fi
