set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -1 gpurun_out/parity.log
timeout -k 10 300 python scripts/launch_perf.py > gpurun_out/launch.log 2>&1 || { tail -30 gpurun_out/launch.log; exit 1; }
grep -v amdgpu.ids gpurun_out/launch.log | head -30; grep -E "j= (20|21|22|23) " gpurun_out/launch.log
timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_iter.json > gpurun_out/bench_iter.log 2>&1 || { tail -30 gpurun_out/bench_iter.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_iter.json'))
r=d['roofline']; print('value', d['value'], 'cells/s; evals/cell', d['evals_per_cell'], '; useful TF', r['useful_tflops_per_gpu'], '; dom', r['kernel'], r['achieved'], 'TF'); print(r['kernels_ms'])"
timeout -k 10 300 python scripts/round_perf.py > gpurun_out/round.log 2>&1 || { tail -30 gpurun_out/round.log; exit 1; }
grep -v amdgpu.ids gpurun_out/round.log
