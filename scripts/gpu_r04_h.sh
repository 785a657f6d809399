# round 4: n x n (OI_DEDUP=0) divergence diagnostic on the day cells with long fits
set -o pipefail
mkdir -p gpurun_out/r04
for c in 37; do
  timeout -k 10 400 python3 scratch/cell_diverge.py $c 0 >> gpurun_out/r04/diverge_h.txt 2>&1 || { tail -20 gpurun_out/r04/diverge_h.txt; exit 1; }
done
cat gpurun_out/r04/diverge_h.txt
