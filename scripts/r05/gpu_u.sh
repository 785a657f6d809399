# round 5: k_stebz Sturm steps with v_rcp_f64 + Newton (no VCC-serialised
# division) at 1 / 2 / 4 (default) / 8 points per sweep: probe timings and
# accuracy; Nystrom tests and line
set -o pipefail
D=gpurun_out/r05/u; mkdir -p $D
for b in eigh_probe_p1 eigh_probe_p2 eigh_probe eigh_probe_p8; do
  timeout -k 10 180 tools/$b 928 64 > $D/$b.txt 2>&1 || { cat $D/$b.txt; exit 1; }
  echo "$b: $(tr '\n' ' ' < $D/$b.txt)"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); s=d['roofline']['stages_ms']
print('new', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:9]})"
