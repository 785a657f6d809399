#!/bin/bash
# round 3: even-step diagonal pre-update (presyrk) -- parity, configs 1/2, the day, SQ PMC on the probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/r03j
mkdir -p $D
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py tests/test_gpu_session.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload predict --steps 50 --warmup 5 > $D/bench_config2.json 2> $D/bench_config2.err || { tail -5 $D/bench_config2.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench_config2.json'));print('config2', d['value'], d['roofline']['kernels_ms'])"
timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 > $D/bench_config1.json 2> $D/bench_config1.err || { tail -5 $D/bench_config1.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench_config1.json'));print('config1', d['value'], d['ms_per_step'], d['cpu_baseline'].get('value'))"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -5 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS --kernel-trace -d $D/pmcS -o run --output-format csv -- python3 scripts/quick_perf.py > $D/pmc_run.log 2>&1 || { tail -5 $D/pmc_run.log; exit 1; }
python3 scripts/pmc_kernels.py $D/pmcS > $D/pmc_sq.txt && cut -c1-300 $D/pmc_sq.txt | head -5
rm -rf $D/pmcS
