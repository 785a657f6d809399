#!/bin/bash
# round 3: fold epilogue v2 (LDS-packed Winv) -- parity, then A/B per-kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03ab2
mkdir -p $D
OI_FOLD=1 timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fold or golden or boundary" --timeout 150 --timeout-method thread > $D/parity.log 2>&1
rc=$?; tail -3 $D/parity.log; [ $rc -eq 0 ] || exit $rc
OI_FOLD=1 timeout -k 10 120 python3 scripts/r03/ab_probe.py fold > $D/ab.txt 2>&1 &&
OI_FOLD=0 timeout -k 10 120 python3 scripts/r03/ab_probe.py percol >> $D/ab.txt 2>&1 &&
OI_FOLD=1 OI_LIB=build_exp/liboi_noepi.so timeout -k 10 120 python3 scripts/r03/ab_probe.py noepi >> $D/ab.txt 2>&1
rc=$?; grep "\[" $D/ab.txt; exit $rc
