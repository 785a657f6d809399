#!/bin/bash
# round 3: Nystrom fit session -- parity vs the one-shot fit, the nystrom bench
# through the session (and one-shot for comparison); config-1 latency timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r03g
mkdir -p $D
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_nystrom.py -m gpu -x -v --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $D/gputests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py --workload nystrom --steps 20 --warmup 2 > $D/bench_nystrom_session.json 2> $D/bench_nystrom_session.err || { tail -20 $D/bench_nystrom_session.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench_nystrom_session.json'));print('session', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'], d['cpu_baseline'].get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/single_trace -o run --output-format csv -- python3 scripts/single_latency.py 200 8 > $D/single_latency.json 2> $D/single_latency.err || { tail -20 $D/single_latency.err; exit 1; }
cat $D/single_latency.json | head -40
python3 scripts/trace_summary.py $D/single_trace > $D/single_trace_summary.txt; head -30 $D/single_trace_summary.txt
find $D/single_trace -name "*kernel_stats.csv" -exec cp {} $D/single_kernel_stats.csv \;
