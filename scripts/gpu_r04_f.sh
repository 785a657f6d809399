# round 4: Nystrom eigensolver v4 (incremental T, batched trailing-update
# loads, unrolled panel corrections) + T3 on the bench day's cells
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests_f.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests_f.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests_f.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out gpurun_out/r04/bench_nystrom_f.json > gpurun_out/r04/bench_nystrom_f.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom_f.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04/bench_nystrom_f.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_day_fits.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r04/day_fits_f.log 2>&1
rc=$?
grep -v "^E  \|amdgpu.ids" gpurun_out/r04/day_fits_f.log | tail -60
exit $rc
