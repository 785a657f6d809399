"""Summary of a rocprofv3 kernel trace: busy/idle time of the GPU, inter-kernel
gaps and per-kernel duration statistics (the raw trace is too big to keep)."""
import csv, glob, os, sys
from collections import defaultdict

import numpy as np

rows = []
for f in glob.glob(os.path.join(sys.argv[1], '**', '*kernel_trace.csv'), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
st = np.array([int(r['Start_Timestamp']) for r in rows])
en = np.array([int(r['End_Timestamp']) for r in rows])
names = [r['Kernel_Name'].split('(')[0] for r in rows]
busy, cs, ce = 0, st[0], en[0]
for s, e in zip(st[1:], en[1:]):
    if s > ce:
        busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
span = en.max() - st.min()
print(f"dispatches {len(rows)} span {span / 1e9:.3f} s busy {busy / 1e9:.3f} s idle {1 - busy / span:.4f}")
d = defaultdict(list)
gap = defaultdict(list)
for i, (n, s, e) in enumerate(zip(names, st, en)):
    d[n].append(e - s)
    if i:
        gap[n].append(max(0, s - en[i - 1]))
for k in sorted(d, key=lambda k: -sum(d[k])):
    v = np.array(d[k]) / 1e3
    g = np.array(gap[k]) / 1e3 if gap[k] else np.zeros(1)
    print(f"{k:32s} n={len(v):7d} total={v.sum() / 1e6:8.3f}s mean={v.mean():9.1f}us p50={np.median(v):9.1f}us "
          f"gap_before_mean={g.mean():7.1f}us")
