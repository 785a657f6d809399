#!/bin/bash
# experimental liboi variants for timing A/B (tools only, never shipped):
#   build_exp/liboi_<tag>.so built with extra -D flags on oi_kernels.hip
# usage: scripts/build_exp_lib.sh <tag> "<-DFLAGS>"
set -e
cd "$(dirname "$0")/../optimalinterpolation_amd"
mkdir -p ../build_exp
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=fast $2 -c csrc/oi_kernels.hip -o ../build_exp/oi_kernels_$1.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../build_exp/liboi_$1.so ../build_exp/oi_kernels_$1.o build/cg.o build/cg_abi.o build/oi_engine.o build/oi_day.o build/oi_day_host.o build/oi_nystrom.o build/oi_linalg.o build/oi_svgp.o
