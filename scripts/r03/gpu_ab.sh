#!/bin/bash
# round 3: A/B of the folded pair step against the per-column scheme and two
# timing-only variants (no triangular epilogue / no look-ahead workgroup)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03ab
mkdir -p $D
timeout -k 10 120 python3 scripts/r03/ab_probe.py fold > $D/ab.txt 2>&1 &&
OI_FOLD=0 timeout -k 10 120 python3 scripts/r03/ab_probe.py percol >> $D/ab.txt 2>&1 &&
OI_LIB=build_exp/liboi_noepi.so timeout -k 10 120 python3 scripts/r03/ab_probe.py noepi >> $D/ab.txt 2>&1 &&
OI_LIB=build_exp/liboi_nola.so timeout -k 10 120 python3 scripts/r03/ab_probe.py nola >> $D/ab.txt 2>&1
rc=$?; grep "\[" $D/ab.txt; exit $rc
