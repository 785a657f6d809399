#!/bin/bash
# triangular chunk masks: GPU tests, per-kernel probe and the day, new library vs build_exp/liboi_base.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${1:-masks}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -2 gpurun_out/gputests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python3 scripts/lauum_probe.py || exit 1
OI_LIB=build_exp/liboi_base.so timeout -k 10 150 python3 scripts/lauum_probe.py || exit 1
for v in new base new; do
  if [ $v = base ]; then export OI_LIB=build_exp/liboi_base.so; else unset OI_LIB; fi
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${TAG}_$v.json 2> gpurun_out/ab_${TAG}_$v.err || exit 1
  echo "$v $(grep 'GPU leg' gpurun_out/ab_${TAG}_$v.err)"
done
