# Rehearse the N>1 bench path on one GPU: 2 ranks sharing GPU 0, gloo collectives.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export OI_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --no-cpu-baseline --out gpurun_out/bench_2rank.json > gpurun_out/bench_2rank.log 2>&1 || { tail -40 gpurun_out/bench_2rank.log; exit 1; }
cat gpurun_out/bench_2rank.json
