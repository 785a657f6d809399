# round 5: the pending eigensolver (liboi_pend.so = this tree + branch
# eigh-opt-pending's oi_linalg) on the Nystrom tests and bench, the session's
# cells-per-group cap, and two stream groups on the day
set -o pipefail
D=gpurun_out/r05/e2; mkdir -p $D
P=$PWD/optimalinterpolation_amd/liboi_pend.so
OI_LIB=$P timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/nys_tests_pend.log 2>&1
rc=$?; tail -2 $D/nys_tests_pend.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $D/nys_tests_pend.log | head -60; exit $rc; }
for v in main pend main64 pend64 pend128; do
  case $v in main) L=""; C="";; pend) L=$P; C="";; main64) L=""; C=64;; pend64) L=$P; C=64;; pend128) L=$P; C=128;; esac
  unset OI_NYS_CAP; [ -n "$C" ] && export OI_NYS_CAP=$C
  OI_LIB=$L timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nys_$v.json > $D/nys_$v.log 2>&1 || { tail -20 $D/nys_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/nys_$v.json')); s=d['roofline']['stages_ms']
print('$v', d['value'], d['evals_per_cell'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:5]})"
done
unset OI_NYS_CAP
for g in 1 2; do
  OI_GROUPS=$g timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --timed-profile off --no-cpu-baseline --parity-cells 4 --out $D/day_g$g.json > $D/day_g$g.log 2>&1 || { tail -20 $D/day_g$g.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/day_g$g.json')); print('groups $g', d['value'], d['timed_s'], d['parity']['pass'])"
done
OI_PANEL4_MINJ=2 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 4 --out $D/day_minj2.json > $D/day_minj2.log 2>&1 || { tail -20 $D/day_minj2.log; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 4 --out $D/day_default.json > $D/day_default.log 2>&1 || { tail -20 $D/day_default.log; exit 1; }
python3 -c "
import json
for f in ('minj2', 'default'):
    d=json.load(open('$D/day_' + f + '.json')); r=d['roofline']; print(f, d['value'], r['frac'], {k: round(v) for k, v in r['kernels_ms'].items()})"
