# round 5: eigensolver probes (OI_SY_S widths, the pending round-4 version),
# the GPU suite on the tree without k_build (generated covariance tiles), and
# the day A/B against the round-4 kernels (liboi_base.so), back to back
set -o pipefail
D=gpurun_out/r05/c; mkdir -p $D
for s in 8 16 32; do
  OI_SY_S=$s timeout -k 10 120 tools/eigh_probe 928 32 > $D/eigh_probe_s$s.txt 2>&1 || { cat $D/eigh_probe_s$s.txt; exit 1; }
  echo "S=$s: $(head -1 $D/eigh_probe_s$s.txt)"
done
timeout -k 10 120 tools/eigh_probe_pend 928 32 > $D/eigh_probe_pend.txt 2>&1 || { cat $D/eigh_probe_pend.txt; exit 1; }
echo "pend: $(head -1 $D/eigh_probe_pend.txt)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fit_large and not day_fits" > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $D/gputests.log | tail -6; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $D/gputests.log | head -120; exit $rc; }
for leg in new base new base; do
  if [ $leg = base ]; then export OI_LIB=$PWD/optimalinterpolation_amd/liboi_base.so; else unset OI_LIB; fi
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 8 --out $D/day_$leg.json > $D/day_$leg.log 2>&1 || { tail -20 $D/day_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/day_$leg.json')); r=d['roofline']
print('$leg', d['value'], r['kernel'], r['frac'], {k: round(v) for k, v in r['kernels_ms'].items()}, d['parity']['pass'], d['parity']['max_rel_fs'])"
done
