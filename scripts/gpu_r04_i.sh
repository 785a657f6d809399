# round 4: per-panel sytrd with GEMM trailing update; T3 with the statistical rules
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/eigh_probe 928 32 > gpurun_out/r04/eigh_probe_i.txt 2>&1 || { cat gpurun_out/r04/eigh_probe_i.txt; exit 1; }
cat gpurun_out/r04/eigh_probe_i.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests_i.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests_i.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests_i.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out gpurun_out/r04/bench_nystrom_i.json > gpurun_out/r04/bench_nystrom_i.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom_i.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04/bench_nystrom_i.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
OI_T3_DUMP=gpurun_out/r04/t3 timeout -k 10 900 python -u -m pytest tests/test_gpu_day_fits.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r04/day_fits_i.log 2>&1
rc=$?
grep "OI_DEDUP\|PASSED\|FAILED\|passed\|failed" gpurun_out/r04/day_fits_i.log
exit $rc
