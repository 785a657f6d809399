set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/parity.log 2>&1
rc=$?
tail -40 gpurun_out/parity.log
exit $rc
