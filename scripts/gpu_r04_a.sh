set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm4_probe > gpurun_out/g4probe.txt 2>&1
echo "probe rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_nystrom.py -x -v --timeout 300 --timeout-method thread > gpurun_out/nys_tests.log 2>&1
echo "nys rc=$?"
tail -30 gpurun_out/nys_tests.log
cat gpurun_out/g4probe.txt
