#!/bin/bash
# Nystrom variant: GPU parity tests
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_nystrom.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/nys_tests.log 2>&1
rc=$?
tail -60 gpurun_out/nys_tests.log
exit $rc
