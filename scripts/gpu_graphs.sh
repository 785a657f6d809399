set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
echo "suite: $(tail -n 1 gpurun_out/gpu_tests.log)"
for g in 1 0; do
  OI_GRAPHS=$g timeout -k 10 300 python bench.py --workload single --steps 5 --warmup 1 --no-cpu-baseline --out gpurun_out/b1.json > gpurun_out/b1.log 2>&1 || { tail -20 gpurun_out/b1.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b1.json')); print('OI_GRAPHS=$g config1 ms/cell', d['ms_per_step'])"
  OI_GRAPHS=$g timeout -k 10 600 python bench.py --workload dayshard --steps 1 --warmup 0 --no-cpu-baseline --out gpurun_out/b2.json > gpurun_out/b2.log 2>&1 || { tail -20 gpurun_out/b2.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b2.json')); print('OI_GRAPHS=$g dayshard', d['value'])"
done
