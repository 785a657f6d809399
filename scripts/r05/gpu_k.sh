# round 5: (1) config 1 with the packed inverse read unconditionally (masked):
# fused vs separate diagonal launches; (2) the eigensolver's next reflector
# formed inside k_sy_w (one launch per column fewer): probe, Nystrom tests
# and line; (3) the one-rank RCCL test
set -o pipefail
D=gpurun_out/r05/k; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_parity.py tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
timeout -k 10 120 tools/eigh_probe 928 64 > $D/eigh_probe_64.txt 2>&1 || { cat $D/eigh_probe_64.txt; exit 1; }
echo "probe: $(head -1 $D/eigh_probe_64.txt)"
for leg in fused sep; do
  if [ $leg = sep ]; then export OI_FUSE_DIAG_MIN=2; else unset OI_FUSE_DIAG_MIN; fi
  timeout -k 10 300 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline --out $D/config1_$leg.json > $D/config1_$leg.log 2>&1 || { tail -20 $D/config1_$leg.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/config1_$leg.json')); r=d['roofline']; print('$leg', d['ms_per_step'], {k: round(v, 1) for k, v in r['kernels_ms'].items()})"
done
unset OI_FUSE_DIAG_MIN
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); s=d['roofline']['stages_ms']
print('nystrom', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:6]})"
