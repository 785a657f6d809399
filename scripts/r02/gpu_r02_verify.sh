#!/bin/bash
# end-of-session verification of the committed tree: GPU test suite, smoke(), the driver's exact bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/verify
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; echo "pytest rc $rc"; grep -E "passed|failed" $D/gputests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
