#!/bin/bash
# config 2 (predict-only) and config 1 (single cell): per-launch events in the
# timed region on/off, resident-cell stream groups 1/2/3; the day with events off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab2
for cfg in "on 1" "off 1" "off 2" "off 3" "off 1"; do
  set -- $cfg
  OI_GROUPS=$2 timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --timed-profile $1 \
    --no-cpu-baseline > gpurun_out/ab2/predict_p$1_g$2.json 2> gpurun_out/ab2/predict_p$1_g$2.err || exit 1
  grep "GPU leg" gpurun_out/ab2/predict_p$1_g$2.err
done
timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 > gpurun_out/ab2/single.json 2> gpurun_out/ab2/single.err || exit 1
grep "GPU leg" gpurun_out/ab2/single.err
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --timed-profile off --no-cpu-baseline > gpurun_out/ab2/day_poff.json 2> gpurun_out/ab2/day_poff.err || exit 1
grep "GPU leg" gpurun_out/ab2/day_poff.err
