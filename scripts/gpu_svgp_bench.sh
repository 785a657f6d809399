#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --workload svgp --out gpurun_out/svgp_bench.json > gpurun_out/svgp_bench.log 2>&1 || { tail -30 gpurun_out/svgp_bench.log; exit 1; }
cat gpurun_out/svgp_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/svgp_prof -o svgp --output-format csv -- python bench.py --workload svgp --no-cpu-baseline --no-prime --out gpurun_out/svgp_bench_prof.json > gpurun_out/svgp_prof.log 2>&1 || { tail -30 gpurun_out/svgp_prof.log; exit 1; }
f=$(find /tmp/svgp_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/svgp_kernel_stats.csv
head -4 gpurun_out/svgp_kernel_stats.csv | cut -c1-220
