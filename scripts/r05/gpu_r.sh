# round 5: non-transposed gemv (A -= W' (W r)) on 16-wave workgroups that
# split the columns: Nystrom tests and line
set -o pipefail
D=gpurun_out/r05/r; mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); s=d['roofline']['stages_ms']
print('gemv_n', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:9]})"
