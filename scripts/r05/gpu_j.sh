# round 5: config 1 with the packed inverse read unconditionally (masked) and
# 16-wide (8 in the first packed version), fused and separate diagonal
# launches; the one-rank RCCL test
set -o pipefail
D=gpurun_out/r05/j; mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
for leg in fused sep fused sep; do
  if [ $leg = sep ]; then export OI_FUSE_DIAG_MIN=2; else unset OI_FUSE_DIAG_MIN; fi
  timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline --out $D/config1_$leg.json > $D/config1_$leg.log 2>&1 || { tail -20 $D/config1_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/config1_$leg.json')); r=d['roofline']; print('$leg', d['ms_per_step'], {k: round(v, 1) for k, v in r['kernels_ms'].items()})"
done
