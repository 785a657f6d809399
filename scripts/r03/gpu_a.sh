#!/bin/bash
# round 3, first call: MFMA/VALU co-issue probe, GPU test suite (new session /
# arena tests included), per-kernel timings at fixed sizes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03a
mkdir -p $D
timeout -k 10 120 ./tools/mix_probe > $D/mix_probe.txt 2>&1 && cat $D/mix_probe.txt &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|Error" $D/gputests.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/quick_perf.py > $D/quick_perf.txt 2>&1 && cat $D/quick_perf.txt
