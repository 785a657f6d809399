#!/bin/bash
# round 3: k_chol_panel A' prefetch -- per-column launch times, parity, the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/${RUN:-r03r}
mkdir -p $D
timeout -k 10 200 python3 scripts/r03/launch_per_j.py > $D/lpj.txt 2>&1 || { tail -5 $D/lpj.txt; exit 1; }
grep -E "^(1|15|31) " $D/lpj.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py tests/test_gpu_session.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -5 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
python3 -c "import json;d=json.load(open('$D/bench_day.json'));print('day', d['value'], d['roofline']['frac'], d['roofline']['kernels_ms'], d['parity']['pass'])"
