# round 5: the Nystrom session's cells-per-group cap (more matrices per batched
# eigensolver call), two stream groups on the day, and k_panel_even for the
# j = 0 column (OI_PANEL4_MINJ=2)
set -o pipefail
D=gpurun_out/r05/e2; mkdir -p $D
for C in 32 64 128; do
  OI_NYS_CAP=$C timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nys_cap$C.json > $D/nys_cap$C.log 2>&1 || { tail -20 $D/nys_cap$C.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/nys_cap$C.json')); s=d['roofline']['stages_ms']
print('cap $C', d['value'], d['evals_per_cell'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:5]})"
done
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
