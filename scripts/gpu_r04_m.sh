# round 4, verification of the tree: eigensolver probe, the whole -m gpu suite,
# smoke(), the Nystrom line, the driver's day command (cpu_baseline from the
# day fixture); every GPU step under its own time limit, stop at the first failure
set -o pipefail
D=gpurun_out/r04/verify; mkdir -p $D
timeout -k 10 120 tools/eigh_probe 928 32 > $D/eigh_probe.txt 2>&1 || { cat $D/eigh_probe.txt; exit 1; }
cat $D/eigh_probe.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $D/gputests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out $D/bench_nystrom.json > $D/bench_nystrom.log 2>&1 || { tail -20 $D/bench_nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_nystrom.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
timeout -k 10 560 python3 bench.py --gpus 1 --steps 20 --warmup 5 --out $D/bench_day.json > $D/bench_day.log 2>&1 || { tail -20 $D/bench_day.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench_day.json')); c=d['cpu_baseline']
print('day', d['value'], d['roofline']['kernel'], d['roofline']['frac'], 'cpu', c['value'], c.get('e_cpu_mean_timed_cells'), c.get('fit_time_residual_max_abs'), d['parity'])"
