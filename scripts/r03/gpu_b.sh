#!/bin/bash
# round 3: duplicate non-PD band test + the driver's bench command with the
# timed-cell parity check and a per-cell dump (E(n) refit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03b
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_session.py -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $D/gputests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --dump $D/day_cells.npz > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err; python3 -c "import json;d=json.load(open('$D/bench_day.json'));print(d['value'],d.get('parity'),d['cpu_baseline'].get('value'))"
