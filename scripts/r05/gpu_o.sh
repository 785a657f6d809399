# round 5: tridiagonalisation in two multi-workgroup launches per column
# (k_sy_symv forms the reflector, k_sy_w by rows) vs the committed build
# (liboi_base.so / eigh_probe_base: k_sy_reflect + one-workgroup k_sy_w):
# probe timings and accuracy, Nystrom tests, Nystrom line for both
set -o pipefail
D=gpurun_out/r05/o; mkdir -p $D
for b in eigh_probe eigh_probe_base; do
  timeout -k 10 180 tools/$b 928 64 > $D/$b.txt 2>&1 || { cat $D/$b.txt; exit 1; }
  echo "$b: $(tr '\n' ' ' < $D/$b.txt)"
done
timeout -k 10 120 tools/eigh_probe 200 16 > $D/eigh_probe_200.txt 2>&1 || { cat $D/eigh_probe_200.txt; exit 1; }
echo "M=200: $(tr '\n' ' ' < $D/eigh_probe_200.txt)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
for leg in new base; do
  if [ $leg = base ]; then export OI_LIB=$PWD/optimalinterpolation_amd/liboi_base.so; else unset OI_LIB; fi
  timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom_$leg.json > $D/nystrom_$leg.log 2>&1 || { tail -20 $D/nystrom_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/nystrom_$leg.json')); s=d['roofline']['stages_ms']
print('$leg', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:8]})"
done
