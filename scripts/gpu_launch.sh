set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/launch_perf.py > gpurun_out/launch.log 2>&1 || { tail -30 gpurun_out/launch.log; exit 1; }
grep -v amdgpu.ids gpurun_out/launch.log
