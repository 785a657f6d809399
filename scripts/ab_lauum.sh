set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
OI_LAUUM=1 timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity1.log 2>&1 || { tail -40 gpurun_out/parity1.log; exit 1; }
tail -1 gpurun_out/parity.log gpurun_out/parity1.log
for v in 0 1 0 1; do
OI_LAUUM=$v timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_ab$v.json > gpurun_out/bench_ab.log 2>&1 || { tail -30 gpurun_out/bench_ab.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_ab$v.json'))
r=d['roofline']; print('OI_LAUUM=$v value', d['value'], 'lauum ms', r['kernels_ms']['k_lauum_grad'])"
done
