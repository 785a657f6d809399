#!/bin/bash
# round 3: 4-wave diagonal factor -- stage probe, parity, config 1/2, the day
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
D=gpurun_out/${RUN:-r03l}
mkdir -p $D
timeout -k 10 60 ./tools/diag_engine_probe > $D/probe4w.txt 2>&1 || { cat $D/probe4w.txt; exit 1; }
OI_DIAG=16 timeout -k 10 60 ./tools/diag_engine_probe > $D/probe16.txt 2>&1 || { cat $D/probe16.txt; exit 1; }
cat $D/probe4w.txt $D/probe16.txt
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py tests/test_gpu_session.py tests/test_gpu_gpr_surface.py -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputests.log 2>&1
rc=$?; tail -3 $D/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 > $D/bench_config1.json 2> $D/bench_config1.err || { tail -5 $D/bench_config1.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench_config1.json'));print('config1', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --workload predict --steps 50 --warmup 5 > $D/bench_config2.json 2> $D/bench_config2.err || { tail -5 $D/bench_config2.err; exit 1; }
python3 -c "import json;d=json.load(open('$D/bench_config2.json'));print('config2', d['value'], d['roofline']['kernels_ms'])"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --parity-cells 24 --no-cpu-baseline > $D/bench_day.json 2> $D/bench_day.err || { tail -5 $D/bench_day.err; exit 1; }
grep "GPU leg" $D/bench_day.err
python3 -c "import json;d=json.load(open('$D/bench_day.json'));print('day', d['value'], d['roofline']['frac'], d['roofline']['kernels_ms'], d['parity']['pass'])"
