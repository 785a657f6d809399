#!/bin/bash
# round 3: LDS re-stride of post_right / post_left -- parity, per-kernel times,
# SQ PMC pass (bank conflicts, MFMA busy) on the fixed-size probe, then the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r03c
mkdir -p $D
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/quick_perf.py > $D/quick_perf.txt 2>&1 && grep -E "SMLII|panel|lauum|chol" $D/quick_perf.txt || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --kernel-trace -d $D/pmcS -o run --output-format csv -- python3 scripts/quick_perf.py > $D/pmc_run.log 2>&1 || { tail -5 $D/pmc_run.log; exit 1; }
python3 scripts/pmc_kernels.py $D/pmcS > $D/pmc_sq.txt && cut -c1-220 $D/pmc_sq.txt | head -12
rm -rf $D/pmcS
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 0 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -20 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err; python3 -c "import json;d=json.load(open('$D/bench_day.json'));r=d['roofline'];print(r['frac'],r['kernels_ms'],r['gemm_kernels'])"
