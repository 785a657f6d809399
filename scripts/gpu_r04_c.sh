# round 4: config-4 share runs (depth 8 and all-in-flight), full GPU test suite
set -o pipefail
mkdir -p gpurun_out/r04
DEPTH=20 bash scripts/r04/gpu_shares.sh > gpurun_out/r04/shares_d20.txt 2>&1 || { tail -20 gpurun_out/r04/shares_d20.txt; exit 1; }
DEPTH=8 bash scripts/r04/gpu_shares.sh > gpurun_out/r04/shares_d8.txt 2>&1 || { tail -20 gpurun_out/r04/shares_d8.txt; exit 1; }
tail -30 gpurun_out/r04/shares_d20.txt
tail -12 gpurun_out/r04/shares_d8.txt
