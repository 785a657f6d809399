# round 4: Nystrom eigensolver v3 (column-group symv, CholQR2 panels, spread
# stebz/stein) tests + bench; T3 on the bench day's own cells (OI_DEDUP 1/0)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/nys_tests_e.log 2>&1 || { tail -30 gpurun_out/r04/nys_tests_e.log; exit 1; }
tail -2 gpurun_out/r04/nys_tests_e.log
timeout -k 10 600 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out gpurun_out/r04/bench_nystrom_e.json > gpurun_out/r04/bench_nystrom_e.log 2>&1 || { tail -20 gpurun_out/r04/bench_nystrom_e.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04/bench_nystrom_e.json')); print('nystrom', d['value'], d['evals_per_cell'], d['roofline']['kernel'], d['roofline']['stages_ms'])"
if [ -f tests/golden/day_ref_fits.npz ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_day_fits.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/r04/day_fits_e.log 2>&1 || { tail -40 gpurun_out/r04/day_fits_e.log; exit 1; }
  tail -40 gpurun_out/r04/day_fits_e.log
fi
