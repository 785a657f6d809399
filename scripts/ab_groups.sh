set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -m pytest tests/test_gpu_parity.py tests/test_gpu_fit.py -x -q -m gpu > gpurun_out/parity.log 2>&1 || { tail -40 gpurun_out/parity.log; exit 1; }
tail -n 1 gpurun_out/parity.log
for v in 2 1 3; do
OI_GROUPS=$v timeout -k 10 400 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/bench_g$v.json > gpurun_out/bench_g.log 2>&1 || { tail -30 gpurun_out/bench_g.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench_g$v.json'))
r=d['roofline']; print('OI_GROUPS=$v value', d['value'], r['kernels_ms'])"
done
