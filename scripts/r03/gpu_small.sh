#!/bin/bash
# round 3: configs 1 and 2 with the folded pair step on and off (same box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
D=gpurun_out/r03small
mkdir -p $D
for f in 0 1; do
  OI_FOLD=$f timeout -k 10 200 python3 bench.py --workload single --steps 20 --warmup 3 --no-cpu-baseline > $D/single_f$f.json 2> $D/single_f$f.err || { tail -5 $D/single_f$f.err; exit 1; }
  OI_FOLD=$f timeout -k 10 200 python3 bench.py --workload predict --steps 20 --warmup 3 --no-cpu-baseline > $D/predict_f$f.json 2> $D/predict_f$f.err || { tail -5 $D/predict_f$f.err; exit 1; }
done
for f in 0 1; do python3 -c "import json;a=json.load(open('$D/single_f$f.json'));b=json.load(open('$D/predict_f$f.json'));print('fold=$f','single',a['value'],a['ms_per_step'],'predict',b['value'],b['ms_per_step'])"; done
