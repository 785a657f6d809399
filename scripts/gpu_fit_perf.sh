set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/quick_perf.py > gpurun_out/perf.log 2>&1 ; rc1=$?
cat gpurun_out/perf.log
[ $rc1 -ne 0 ] && exit $rc1
timeout -k 10 600 python -m pytest tests/test_gpu_fit.py -x -q -m gpu > gpurun_out/fit.log 2>&1
rc=$?
tail -30 gpurun_out/fit.log
exit $rc
