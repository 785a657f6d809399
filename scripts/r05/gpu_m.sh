# round 5: eigensolver orthogonalisation on 128-column blocks (two-level
# BCGS2) vs panel-wise BCGS2 (OI_ORTH_BLOCK=32): probe timings and accuracy,
# Nystrom tests, Nystrom line for both
set -o pipefail
D=gpurun_out/r05/m; mkdir -p $D
for ob in 32 128 256; do
  OI_ORTH_BLOCK=$ob timeout -k 10 180 tools/eigh_probe 928 64 > $D/eigh_probe_ob$ob.txt 2>&1 || { cat $D/eigh_probe_ob$ob.txt; exit 1; }
  echo "ob $ob: $(tr '\n' ' ' < $D/eigh_probe_ob$ob.txt)"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
for leg in 128 32; do
  OI_ORTH_BLOCK=$leg timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom_ob$leg.json > $D/nystrom_ob$leg.log 2>&1 || { tail -20 $D/nystrom_ob$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/nystrom_ob$leg.json')); s=d['roofline']['stages_ms']
print('ob $leg', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:8]})"
done
