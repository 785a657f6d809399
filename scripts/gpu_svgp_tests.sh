#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_svgp.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/svgp_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|rel|Error|assert|passed|failed" gpurun_out/svgp_tests.log | tail -30
exit $rc
