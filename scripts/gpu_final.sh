# End-of-round check: all GPU tests, smoke, default bench, rocprofv3 kernel stats of the same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 900 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('bench', d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-prime --out gpurun_out/bench_prof.json > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
cp /tmp/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null || cp $(find /tmp/prof -name "*kernel_stats.csv" | head -1) gpurun_out/kernel_stats.csv
grep -E "panel_even" gpurun_out/kernel_stats.csv | cut -c1-160
python -c "import json;d=json.load(open('gpurun_out/bench_prof.json'));print('under rocprof', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['launches'])"
