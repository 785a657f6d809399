# round 5, end-of-session verification of the committed tree, in two calls
# (each under gpurun's 1200 s): PART=tests -- the whole -m gpu suite (T3 day
# fits on the extended fixture included); PART=bench -- smoke() and the
# driver's exact bench command.  Every GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r05/verify; mkdir -p $D
if [ "${PART:-tests}" = tests ]; then
  OI_T3_DUMP=$D/t3 timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $D/gputests.log 2>&1
  rc=$?; grep -E "passed|failed" $D/gputests.log | tail -2; grep -E "OI_DEDUP=" $D/gputests.log | head -20; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $D/gputests.log | head; exit $rc; }
else
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
  tail -1 $D/smoke.log
  timeout -k 10 700 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$D/bench_day.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline']
print('day', d['value'], r['kernel'], r['frac'], r['traffic'], 'cpu', c['value'], d['parity']['pass'], d['ranks_seen'])"
fi
