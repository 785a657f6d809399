#!/bin/bash
# tools/eigh_probe: the probe + oi_linalg.hip
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off \
  eigh_probe.cpp ../optimalinterpolation_amd/csrc/oi_linalg.hip -o eigh_probe
