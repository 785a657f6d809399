set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for g in 2 1; do
  OI_GROUPS=$g timeout -k 10 600 python bench.py --no-cpu-baseline --out gpurun_out/bench_g.json > gpurun_out/bench_g.log 2>&1 || { tail -30 gpurun_out/bench_g.log; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_g.json')); print('OI_GROUPS=$g value', d['value'], 'evals', d['evals_per_cell'], 'dom', d['roofline']['achieved'])"
done
