# round 5: k_potrf_tile's inverse in registers (it was in scratch) and k_stebz
# multisection (4 Sturm counts per sweep): probe timings / accuracy, Nystrom
# tests and line, kernel stats of the line
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r05/t; mkdir -p $D
for a in "928 64" "200 16" "1500 8"; do
  timeout -k 10 180 tools/eigh_probe $a > $D/eigh_probe_${a// /x}.txt 2>&1 || { cat $D/eigh_probe_${a// /x}.txt; exit 1; }
  echo "$a: $(tr '\n' ' ' < $D/eigh_probe_${a// /x}.txt)"
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_nystrom.py -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1
rc=$?; tail -1 $D/tests.log; [ $rc -eq 0 ] || { tail -40 $D/tests.log; exit $rc; }
timeout -k 10 400 python3 bench.py --workload nystrom --steps 10 --warmup 2 --no-cpu-baseline --out $D/nystrom.json > $D/nystrom.log 2>&1 || { tail -20 $D/nystrom.log; exit 1; }
python3 -c "
import json; d=json.load(open('$D/nystrom.json')); s=d['roofline']['stages_ms']
print('new', d['value'], {k: round(v) for k, v in sorted(s.items(), key=lambda x: -x[1])[:9]})"
TAG=t/prof bash scripts/r05/gpu_s.sh | head -16
