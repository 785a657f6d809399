#!/bin/bash
# round 3: micro-variants (streaming k_build stores, one Newton step in the
# diagonal potrf) against the default build: per-kernel times and config 1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03micro
mkdir -p $D
timeout -k 10 120 python3 scripts/r03/ab_probe.py default > $D/ab.txt 2>&1 &&
OI_LIB=build_exp/liboi_nt.so timeout -k 10 120 python3 scripts/r03/ab_probe.py build_nt >> $D/ab.txt 2>&1 &&
OI_LIB=build_exp/liboi_newton1.so timeout -k 10 120 python3 scripts/r03/ab_probe.py newton1 >> $D/ab.txt 2>&1 &&
timeout -k 10 200 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline > $D/single_default.json 2> $D/single_default.err &&
OI_LIB=build_exp/liboi_newton1.so timeout -k 10 200 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline > $D/single_newton1.json 2> $D/single_newton1.err
rc=$?; grep "\[" $D/ab.txt; for f in default newton1; do python3 -c "import json;a=json.load(open('$D/single_$f.json'));print('$f single',a['value'],a['ms_per_step'],a['evals_per_cell'])"; done; exit $rc
