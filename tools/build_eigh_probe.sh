#!/bin/bash
# tools/eigh_probe: oi_linalg.hip with the k_sytrd phase stamps + the probe
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 -ffp-contract=off -DOI_SYTRD_TIMING \
  eigh_probe.cpp ../optimalinterpolation_amd/csrc/oi_linalg.hip -o eigh_probe
