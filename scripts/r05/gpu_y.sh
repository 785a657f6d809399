# round 5: SVGP throughput vs threads per cell and cells per launch (one
# 1024-thread workgroup per CU at 256 cells; smaller workgroups, more cells)
set -o pipefail
D=gpurun_out/r05/y; mkdir -p $D
for cfg in "1024 256" "512 512" "256 1024" "512 256" "1024 512"; do
  set -- $cfg
  OI_SVGP_THREADS=$1 timeout -k 10 300 python3 bench.py --workload svgp --svgp-cells $2 --steps 1 --warmup 1 --no-cpu-baseline --out $D/svgp_t$1_c$2.json > $D/svgp_t$1_c$2.log 2>&1 || { tail -20 $D/svgp_t$1_c$2.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/svgp_t$1_c$2.json')); print('threads $1 cells $2:', d['value'], 'cells/s', d['ms_per_step'], 'ms', d.get('failed_cells'))"
done
