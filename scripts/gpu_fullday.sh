set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python scripts/fullday_probe.py 0 4096 > gpurun_out/fullday.log 2>&1 || { tail -20 gpurun_out/fullday.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fullday.log
