# round 4: Nystrom tests + bench after the cluster-aware eigenvector step; config-4 shares
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests_d.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests_d.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests_d.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 20 --warmup 2 --out gpurun_out/r04/bench_nystrom_d.json > gpurun_out/r04/bench_nystrom_d.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom_d.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04/bench_nystrom_d.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
DEPTH=20 timeout -k 10 900 bash scripts/r04/gpu_shares.sh > gpurun_out/r04/shares_d20.txt 2>&1 || { tail -20 gpurun_out/r04/shares_d20.txt; exit 1; }
tail -25 gpurun_out/r04/shares_d20.txt
