# round 5: k_panel_even's look-ahead made bitwise equal to k_panel4's and the
# per-round choice of the even-column kernel by launch size (OI_PANEL4_MINWG):
# the GPU suite, the day A/B against the previous commit's build
# (liboi_head.so), and the Nystrom line with its CPU baseline
set -o pipefail
D=gpurun_out/r05/h; mkdir -p $D
H=$PWD/optimalinterpolation_amd/liboi_head.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not fit_large and not day_fits" > $D/gputests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $D/gputests.log | tail -6; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $D/gputests.log | head -120; exit $rc; }
for leg in cur head cur head; do
  if [ $leg = head ]; then export OI_LIB=$H; else unset OI_LIB; fi
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-cells 8 --out $D/day_$leg.json > $D/day_$leg.log 2>&1 || { tail -20 $D/day_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/day_$leg.json')); r=d['roofline']
print('$leg', d['value'], r['kernel'], r['frac'], {k: round(v) for k, v in r['kernels_ms'].items()}, d['rounds']['lt256_gpu_ms'], d['parity']['pass'])"
done
unset OI_LIB
timeout -k 10 500 python3 bench.py --workload nystrom --steps 10 --warmup 2 --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); print('nystrom', d['value'], d['roofline']['kernel'], (d['cpu_baseline'] or {}).get('value'))"
timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --out $D/config1.json > $D/config1.log 2>&1 || { tail -20 $D/config1.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/config1.json')); r=d['roofline']; print('config1', d['value'], d['ms_per_step'], {k: round(v, 1) for k, v in r['kernels_ms'].items()}, (d['cpu_baseline'] or {}).get('value'))"
