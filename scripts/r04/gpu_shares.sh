# config 4 on one GPU: the 8 LPT shares of the 25 km day, back to back, each
# through the same slice/session path as the headline (--steps 20), then the
# 1-GPU whole-day line for the efficiency denominator
set -o pipefail
D=gpurun_out/r04/shares_d${DEPTH:-8}; mkdir -p $D
for k in 0 1 2 3 4 5 6 7; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup 2 --day-shares 8 --share $k --depth ${DEPTH:-8} \
    --no-cpu-baseline --parity-cells 0 --out $D/share_$k.json > $D/share_$k.log 2>&1 || { tail -20 $D/share_$k.log; exit 1; }
  python3 -c "import json; d=json.load(open('$D/share_$k.json')); print($k, d['value'], d['timed_s'], d['config']['cells_per_rank'])"
done
python3 scripts/r04/share_projection.py $D
