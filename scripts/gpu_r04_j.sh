# round 4: eigensolver / oila GEMM with global-space and buffer (bounds-checked) loads
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/eigh_probe 928 32 > gpurun_out/r04/eigh_probe_j.txt 2>&1 || { cat gpurun_out/r04/eigh_probe_j.txt; exit 1; }
cat gpurun_out/r04/eigh_probe_j.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests_j.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests_j.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests_j.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out gpurun_out/r04/bench_nystrom_j.json > gpurun_out/r04/bench_nystrom_j.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom_j.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04/bench_nystrom_j.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
export TMPDIR=/tmp
D=gpurun_out/r04/nys_trace; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- python3 bench.py --workload nystrom --steps 2 --warmup 0 --no-cpu-baseline --out $D/bench.json > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
find $D/t -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
rm -rf $D/t
head -25 $D/kernel_stats.csv | cut -c1-150
