# Per-launch timing of the paired-column scheme, then the default bench (algorithmic roofline).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/launch_perf2.py > gpurun_out/launch2.log 2>&1 || { tail -30 gpurun_out/launch2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/launch2.log | tail -80
timeout -k 10 900 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));r=d['roofline'];print('bench', d['value'], r['kernel'], r['achieved'], r['frac'], r['frac_executed'], r['kernels_ms'], d['cpu_baseline']['value'])"
