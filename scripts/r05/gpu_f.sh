# round 5: packed diagonal factor (L and L^-1 in one 64 x 65 LDS array) and the
# next diagonal tile factored by the panels' look-ahead workgroup (no
# k_diag_factor4w launch past column 0; liboi_f.so): bitwise A/B against the
# previous build (liboi_prev.so, same arithmetic expected); then the current
# tree (+ A' / Vneg preloaded into k_chol_panel's accumulators): the GPU
# suite, the day A/B of the three builds, and the 8-rank self-launched day on
# one GPU (gloo)
set -o pipefail
D=gpurun_out/r05/f; mkdir -p $D
P=$PWD/optimalinterpolation_amd/liboi_prev.so
OI_SMALL=0 OI_LIB=$P timeout -k 10 300 python3 tools/ab_bitwise.py run $D/ab_prev.npz > $D/ab_prev.log 2>&1 || { tail -20 $D/ab_prev.log; exit 1; }
F=$PWD/optimalinterpolation_amd/liboi_f.so
OI_LIB=$F timeout -k 10 300 python3 tools/ab_bitwise.py run $D/ab_new.npz > $D/ab_new.log 2>&1 || { tail -20 $D/ab_new.log; exit 1; }
python3 tools/ab_bitwise.py cmp $D/ab_prev.npz $D/ab_new.npz | tee $D/ab_cmp.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fit_large and not day_fits" > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $D/gputests.log | tail -6; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $D/gputests.log | head -120; exit $rc; }
for leg in cur f prev cur; do
  case $leg in prev) export OI_LIB=$P;; f) export OI_LIB=$F;; *) unset OI_LIB;; esac
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 8 --out $D/day_$leg.json > $D/day_$leg.log 2>&1 || { tail -20 $D/day_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/day_$leg.json')); r=d['roofline']
print('$leg', d['value'], r['kernel'], r['frac'], {k: round(v) for k, v in r['kernels_ms'].items()}, d['parity']['pass'])"
done
unset OI_LIB
OI_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 8 --steps 20 --warmup 2 --no-cpu-baseline --parity-cells 8 --out $D/day_8rank_gloo.json > $D/day_8rank_gloo.log 2>&1 || { tail -30 $D/day_8rank_gloo.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/day_8rank_gloo.json')); print('8 ranks on 1 GPU', d['value'], d['n_gpus'], d['ranks_seen'], d['rank_devices'], d['collective_backend'], d['launcher'], d['config']['cells_total'], d['parity']['pass'])"
