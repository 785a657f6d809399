"""Pool the bench-day T3 results over all 680 fixture cells (the 360 the
literal rules were set on + the round-6 replication sample of 320) from the
GPU dumps of tests/test_gpu_day_fits.py (OI_T3_DUMP), with that file's own
statistical tests.  CPU only:
    python scripts/r06/t3_pooled.py gpurun_out/r06/c16/t3 > profiles/r06/t3_replication/pooled.txt"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'tests'))
from test_gpu_day_fits import order_test, worst_test, rank_test, eval_ratio  # noqa: E402

d = np.load('tests/golden/day_ref_fits.npz')
for dedup in (1, 0):
    g = np.load(os.path.join(sys.argv[1], f'gpu_day_fits_dedup{dedup}.npz'))
    out, nlz_gpu, info = g['out'], g['nlz'], g['info']
    for name, m in (('base 360', d['stratum'] != 3), ('replication 320', d['stratum'] == 3),
                    ('pooled 680', np.ones(len(d['sizes']), bool))):
        nlz, out8, ev = d['nlz'][m], d['out8'][m], d['evals'][m]
        f_env = nlz[:, :4].max(1)
        tol = 1e-8 * np.abs(nlz[:, 0]) + 1e-9
        same = np.array([np.allclose(o, r, rtol=1e-6, atol=0) for o, r in zip(out[m], out8[:, 0])])
        miss = int(np.sum(~same & ~(nlz_gpu[m] <= f_env + tol)))
        miss_ref = int(np.sum(nlz[:, 4] > f_env + tol))
        k, expect, pw = worst_test(nlz_gpu[m], nlz)
        ref_fs = out8[:, 0, 0]
        rel = np.where(np.isfinite(out[m][:, 0]), np.abs(out[m][:, 0] - ref_fs) / np.abs(ref_fs), np.inf)
        rel_ref = np.abs(out8[:, 1:, 0] - ref_fs[:, None]) / np.abs(ref_fs[:, None])
        ko, eo, po = order_test(rel > 1e-6, rel_ref > 1e-6)
        mr, z = rank_test(info[m][:, 3], ev)
        r, lo, hi = eval_ratio(info[m][:, 3], ev.astype(float).mean(1))
        print(f"OI_DEDUP={dedup} {name:16s}: envelope misses GPU {miss} vs held-out run {miss_ref}; "
              f"GPU strict worst of 6 in {k} (expected {expect:.1f}, P = {pw:.3f}); beyond 1e-6 GPU "
              f"{np.mean(rel > 1e-6):.3f} vs reference {np.mean(rel_ref > 1e-6):.3f} "
              f"(per run {np.round(np.mean(rel_ref > 1e-6, 0), 3).tolist()}, P = {po:.3f}); "
              f"evaluations {r:.3f} [{lo:.3f} .. {hi:.3f}], rank z = {z:.2f}")
