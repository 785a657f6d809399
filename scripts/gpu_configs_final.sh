# Config 1 / config 2 / Nystrom bench lines on the final tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload predict --steps 10 --warmup 2 --out gpurun_out/bench_config2.json > gpurun_out/cfg2.log 2>&1 || { tail -20 gpurun_out/cfg2.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_config2.json'));print('config2', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 300 python bench.py --workload single --steps 5 --warmup 1 --out gpurun_out/bench_config1.json > gpurun_out/cfg1.log 2>&1 || { tail -20 gpurun_out/cfg1.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_config1.json'));print('config1', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 400 python bench.py --workload nystrom --out gpurun_out/bench_nystrom.json > gpurun_out/nys.log 2>&1 || { tail -20 gpurun_out/nys.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_nystrom.json'));print('nystrom', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
