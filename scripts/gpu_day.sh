# Day-pipeline GPU tests (smoothing, ball query, gather, two-pass day).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_day.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_day.log 2>&1 || { tail -60 gpurun_out/gpu_day.log; exit 1; }
tail -n 15 gpurun_out/gpu_day.log
