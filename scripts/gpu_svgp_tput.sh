#!/bin/bash
# SVGP kernel throughput over (threads, panels) configurations: SVGP_CFGS="512_1 1024_0 ..."
mkdir -p gpurun_out
if [ -n "$SVGP_PROBE" ]; then
  timeout -k 10 300 python -u tools/svgp_probe.py > gpurun_out/svgp_probe.log 2>&1 || { cat gpurun_out/svgp_probe.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/svgp_probe.log
fi
for cfg in $SVGP_CFGS; do
  set -- $(echo $cfg | tr _ " ")
  OI_SVGP_THREADS=$1 OI_SVGP_PANELS=$2 timeout -k 10 200 python -u tools/svgp_tput.py 200 512 > gpurun_out/svgp_tput.log 2>&1 || { cat gpurun_out/svgp_tput.log; exit 1; }
  echo "panels=$2"; grep threads gpurun_out/svgp_tput.log
done
