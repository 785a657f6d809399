set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fit.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/fit.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/fit.log | tail -8
exit $rc
