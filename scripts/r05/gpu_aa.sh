# round 5: k_gemm128 (and since the second run k_gemm) staged as element pairs (16-byte buffer loads on
# interior chunks, swizzle m ^ 4 (k >> 1)): GEMM probe, eigensolver probe,
# Nystrom tests (the 64 / 128 bitwise test included) and line
set -o pipefail
D=gpurun_out/r05/${TAG:-aa}; mkdir -p $D
for g in 1 0; do OI_GEMM128=$g timeout -k 10 60 tools/gemm_probe 4600 928 32 | sed "s/^/pairs gemm128=$g /" | tee -a $D/gemm_probe.txt; done
timeout -k 10 180 tools/eigh_probe 928 64 > $D/eigh_probe.txt 2>&1 || { cat $D/eigh_probe.txt; exit 1; }
echo "probe: $(tr '\n' ' ' < $D/eigh_probe.txt)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); s=d['roofline']['stages_ms']
print('new', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:9]})"
