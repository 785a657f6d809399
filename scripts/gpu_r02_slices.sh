#!/bin/bash
# round 2: multi-rank HIP test + slice-order / pipeline-depth A/B of the session bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gputests_r02d.log 2>&1
echo "pytest rc $?"; tail -3 gpurun_out/gputests_r02d.log
for cfg in "ordered 1" "ordered 3" "lpt 3"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --slices $1 --depth $2 --no-cpu-baseline > gpurun_out/bench_r02_$1_d$2.json 2> gpurun_out/bench_r02_$1_d$2.err
  rc=$?; echo "bench $cfg rc $rc"; grep "GPU leg" gpurun_out/bench_r02_$1_d$2.err
  [ $rc -eq 0 ] || exit $rc
done
