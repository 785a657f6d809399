set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 900 python bench.py --out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.json
