#!/bin/bash
# round 3: in-region radius query + gather; flag completion; 4-wave diagonal factor
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/${RUN:-r03p}
mkdir -p $D
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_day.py tests/test_gpu_multirank.py tests/test_gpu_nystrom.py tests/test_gpu_svgp.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -5 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
python3 -c "import json;d=json.load(open('$D/bench_day.json'));print('day', d['value'], d['roofline']['frac'], d['roofline']['kernels_ms'], d['parity']['pass'], d['config'].get('neighbour_query'))"
