"""Per-round view of a rocprofv3 kernel trace of the engine (a round starts at
k_build): the GPU span of a round, the kernel time inside it, the idle time
between its kernels and the host gap before the next round."""
import csv
import glob
import os
import sys

import numpy as np

rows = []
for f in glob.glob(os.path.join(sys.argv[1], '**', '*kernel_trace.csv'), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rounds, cur = [], []
for r in rows:
    name = r['Kernel_Name'].split('(')[0]
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if name == 'k_build' and cur:
        rounds.append(cur)
        cur = []
    if name.startswith('k_'):
        cur.append((name, s, e))
if cur:
    rounds.append(cur)
span = np.array([r[-1][2] - r[0][1] for r in rounds]) / 1e3
busy = np.array([sum(e - s for _, s, e in r) for r in rounds]) / 1e3
nk = np.array([len(r) for r in rounds])
hgap = np.array([rounds[i + 1][0][1] - rounds[i][-1][2] for i in range(len(rounds) - 1)] or [0]) / 1e3
print(f"rounds {len(rounds)}  kernels/round {np.median(nk):.0f}")
print(f"GPU span per round   mean {span.mean():8.1f} us  p50 {np.median(span):8.1f} us")
print(f"kernel time / round  mean {busy.mean():8.1f} us  p50 {np.median(busy):8.1f} us")
print(f"idle inside round    mean {(span - busy).mean():8.1f} us  ({(span - busy).mean() / max(nk.mean() - 1, 1):.1f} us per gap)")
print(f"host gap to next     mean {hgap.mean():8.1f} us  p50 {np.median(hgap):8.1f} us")
per = {}
for r in rounds:
    for n, s, e in r:
        per.setdefault(n, []).append((e - s) / 1e3)
for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {n:22s} n={len(v):6d} mean {np.mean(v):7.2f} us  per round {sum(v) / len(rounds):7.1f} us")
