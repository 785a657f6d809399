# round 4: glds probe, Nystrom (hand-written eigensolver) and parity tests after the prune
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm4_probe > gpurun_out/g4probe.txt 2>&1; echo "probe rc=$?"
timeout -k 10 900 python -u -m pytest tests/test_gpu_nystrom.py tests/test_gpu_parity.py tests/test_gpu_season.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04a_tests.log | tail -60
cat gpurun_out/g4probe.txt
exit $rc
