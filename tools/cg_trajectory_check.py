"""GPU box: nlZ / status of the GPU (both site forms) along the oracle CG trajectory of tools/cg_oracle_trajectory.py."""
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from optimalinterpolation_amd import _lib
d = np.load('tests/golden/day_ref_fits.npz')
t = np.load('profiles/r04/t3/cell37_oracle_trajectory.npz')
c = 37; a, b = d['offs'][c], d['offs'][c + 1]
x = d['x'].reshape(-1, 3)[a:b]; y = d['y'][a:b]; mean = float(d['mean'])
H, F = t['H'], t['F']
for dd in ('1', '0'):
    os.environ['OI_DEDUP'] = dd
    nlz, g, st = _lib.nlml_grad_batch(np.tile(x, (len(H), 1)), np.tile(y, len(H)), np.full(len(y) * len(H), mean),
                                      np.arange(len(H) + 1) * len(y), H)
    rel = np.abs(nlz - F) / np.abs(F)
    print(f"OI_DEDUP={dd}: status counts {np.bincount(st)}, max rel nlZ diff {np.nanmax(rel):.2e}, "
          f"nonfinite {np.sum(~np.isfinite(nlz))}")
    bad = np.flatnonzero(~(rel <= 1e-8))
    for k in bad[:10]:
        print('  eval', k, 'h', np.round(H[k], 4).tolist(), 'gpu', nlz[k], 'oracle', F[k], 'st', st[k])
