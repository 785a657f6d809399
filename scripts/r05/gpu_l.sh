# round 5: oila::gemm on 128 x 128 tiles (k_gemm128) for products with
# m, n >= 128 vs the 64 x 64 kernel (OI_GEMM128=0): Nystrom tests (incl. the
# bitwise A/B test) and the Nystrom line for both, alternating
set -o pipefail
D=gpurun_out/r05/l; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
for leg in wide narrow wide; do
  if [ $leg = narrow ]; then export OI_GEMM128=0; else unset OI_GEMM128; fi
  timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom_$leg.json > $D/nystrom_$leg.log 2>&1 || { tail -20 $D/nystrom_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/nystrom_$leg.json')); s=d['roofline']['stages_ms']
print('$leg', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:8]})"
done
