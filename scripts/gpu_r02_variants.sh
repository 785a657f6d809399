#!/bin/bash
# the notebook variants on the final tree: Nystrom (NB1 cell 5 shape) and SVGP (NB2 cell 5 shape)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/variants
mkdir -p $D
timeout -k 10 400 python3 bench.py --workload nystrom > $D/bench_nystrom.json 2> $D/bench_nystrom.err || { tail -20 $D/bench_nystrom.err; exit 1; }
grep -c value $D/bench_nystrom.json
timeout -k 10 400 python3 bench.py --workload svgp > $D/bench_svgp.json 2> $D/bench_svgp.err || { tail -20 $D/bench_svgp.err; exit 1; }
grep -c value $D/bench_svgp.json
