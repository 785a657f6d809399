#!/bin/bash
# Round-6 end-of-round check of the committed tree, the driver's own commands:
# the whole -m gpu suite (T1 / T3 arrays dumped and compared bit for bit with
# profiles/r06/t3_replication/{t1,t3}, the 680 day cells), smoke(), and `python3 bench.py --gpus 1 --steps 20
# --warmup 5`; outputs to gpurun_out/verify_$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-r06}
D=gpurun_out/verify_$TAG
mkdir -p $D
OI_T1_DUMP=$D/t1 OI_T3_DUMP=$D/t3 timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed" $D/gputests.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/gputests.log | head; exit $rc; }
python3 scripts/r06/cmp_dumps.py $D/t1 profiles/r06/t3_replication/t1 > $D/cmp_t1.txt && python3 scripts/r06/cmp_dumps.py $D/t3 profiles/r06/t3_replication/t3 > $D/cmp_t3.txt
rc=$?; tail -2 $D/cmp_t3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
rc=$?; tail -1 $D/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $D/bench_day.json > $D/bench_day.log 2>&1
rc=$?; tail -c 400 $D/bench_day.json; echo; [ $rc -eq 0 ] || { tail -20 $D/bench_day.log; exit $rc; }
