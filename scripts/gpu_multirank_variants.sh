# Rehearse the N>1 paths of the notebook-variant workloads and the default day on one GPU
# (2 ranks sharing GPU 0, gloo collectives).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export OI_DIST_BACKEND=gloo
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29541 bench.py --gpus 2 --workload svgp --svgp-cells 16 --svgp-iters 500 --out gpurun_out/svgp_2rank.json > gpurun_out/svgp_2rank.log 2>&1 || { tail -30 gpurun_out/svgp_2rank.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/svgp_2rank.json'));print('svgp 2 ranks', d['value'], d['n_gpus'], d['config']['cells_per_step'])"
timeout -k 10 300 $R --master-port 29542 bench.py --gpus 2 --workload nystrom --nys-cells 4 --out gpurun_out/nys_2rank.json > gpurun_out/nys_2rank.log 2>&1 || { tail -30 gpurun_out/nys_2rank.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/nys_2rank.json'));print('nystrom 2 ranks', d['value'], d['n_gpus'], d['config']['cells_per_step'])"
timeout -k 10 600 $R --master-port 29543 bench.py --gpus 2 --no-cpu-baseline --out gpurun_out/bench_2rank.json > gpurun_out/bench_2rank.log 2>&1 || { tail -30 gpurun_out/bench_2rank.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_2rank.json'));print('day 2 ranks', d['value'], d['n_gpus'], d['scaling'])"
