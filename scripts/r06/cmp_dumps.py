"""Bitwise comparison of two sets of T1 / T3 GPU dumps (tests/test_gpu_day_t1.py
OI_T1_DUMP, tests/test_gpu_day_fits.py OI_T3_DUMP): a kernel / finalize change
that is meant to keep every non-degenerate result bit for bit is checked on the
360 bench-day cells' objective values and full fits.
Usage: python scripts/r06/cmp_dumps.py NEW_DIR OLD_DIR"""
import glob
import os
import sys

import numpy as np

new, old = sys.argv[1], sys.argv[2]
bad = 0
for f in sorted(glob.glob(os.path.join(old, '*.npz'))):
    g = os.path.join(new, os.path.basename(f))
    if not os.path.exists(g):
        print('missing', g)
        bad += 1
        continue
    a, b = np.load(f), np.load(g)
    for k in a.files:
        same = np.array_equal(a[k], b[k], equal_nan=True)
        print(f"{os.path.basename(f)}:{k} {'bitwise equal' if same else 'DIFFERS'}")
        bad += 0 if same else 1
sys.exit(1 if bad else 0)
