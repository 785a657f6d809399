#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/svgp_probe.py > gpurun_out/svgp_probe.log 2>&1; rc=$?
cat gpurun_out/svgp_probe.log | grep -v amdgpu.ids
exit $rc
