# round 4: eigh phase probe; cell-37 n x n vs site-form diagnostic; T3 dumps
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 tools/eigh_probe 928 32 > gpurun_out/r04/eigh_probe_g.txt 2>&1 || { cat gpurun_out/r04/eigh_probe_g.txt; exit 1; }
cat gpurun_out/r04/eigh_probe_g.txt
timeout -k 10 300 python3 scratch/cell37_gpu.py > gpurun_out/r04/cell37_g.txt 2>&1 || { tail -20 gpurun_out/r04/cell37_g.txt; exit 1; }
cat gpurun_out/r04/cell37_g.txt
OI_T3_DUMP=gpurun_out/r04/t3 timeout -k 10 900 python -u -m pytest tests/test_gpu_day_fits.py -q -s --timeout 600 --timeout-method thread -k "evaluation_ratio" > gpurun_out/r04/day_fits_g.log 2>&1
grep "OI_DEDUP" gpurun_out/r04/day_fits_g.log
ls gpurun_out/r04/t3
