#!/bin/bash
# round 3: per-(kernel, j) launch totals of the day (the profiled pass of the driver's command)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03byj
mkdir -p $D
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline --dump $D/day.npz > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err; ls -la $D
