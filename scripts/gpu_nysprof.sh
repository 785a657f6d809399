#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/nys_prof -o nys --output-format csv -- python bench.py --workload nystrom --steps 1 --warmup 0 --no-cpu-baseline --no-prime --out gpurun_out/nys_bench_prof.json > gpurun_out/nys_prof.log 2>&1 || { tail -30 gpurun_out/nys_prof.log; exit 1; }
f=$(find /tmp/nys_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/nys_kernel_stats.csv
cat gpurun_out/nys_bench_prof.json
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/nys_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:22]:
    print(f"{float(r['TotalDurationNs'])/1e6:10.1f} ms {float(r['TotalDurationNs'])/tot*100:5.1f}% {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
print('total', tot/1e6, 'ms')
PY
