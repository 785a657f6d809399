#!/bin/bash
# post-form panels (no k_scale): GPU parity suite, then config 2 / config 1 / the day, post vs P-form
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/post
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/post/gputests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" gpurun_out/post/gputests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/post/gputests.log | head -20; exit $rc; }
for pf in 0 1 0 1; do
  OI_PFORM=$pf timeout -k 10 200 python3 bench.py --workload predict --steps 50 --warmup 5 --no-cpu-baseline \
    > gpurun_out/post/predict_pf$pf.json 2> gpurun_out/post/predict_pf$pf.err || exit 1
  echo "pform $pf"; grep "GPU leg" gpurun_out/post/predict_pf$pf.err
done
for pf in 0 1; do
  OI_PFORM=$pf timeout -k 10 200 python3 bench.py --workload single --steps 10 --warmup 2 \
    > gpurun_out/post/single_pf$pf.json 2> gpurun_out/post/single_pf$pf.err || exit 1
  echo "pform $pf"; grep "GPU leg" gpurun_out/post/single_pf$pf.err
done
for pf in 0 1; do
  OI_PFORM=$pf timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/post/day_pf$pf.json 2> gpurun_out/post/day_pf$pf.err || exit 1
  echo "pform $pf"; grep "GPU leg" gpurun_out/post/day_pf$pf.err
done
