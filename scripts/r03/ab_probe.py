"""Per-kernel times of one SMLII evaluation over fixed batches (256 x n=3000,
512 x n=1600, 1000 x n=500), for A/B runs of build variants (OI_LIB) or
environment switches (OI_FOLD, ...).  Prints one line per kernel."""
import os, sys, time
import numpy as np
sys.path.insert(0, '.')
from optimalinterpolation_amd import _lib, synthetic
tag = sys.argv[1] if len(sys.argv) > 1 else 'default'
for n, nc in [(3000, 256), (1600, 512), (500, 1000)]:
    cells = synthetic.make_cells([n] * nc, seed=3)
    h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
    mX = np.full(len(cells.z), cells.mean)
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
    best = None
    for rep in range(3):
        _lib.profile_reset()
        _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True)
        pj = _lib.profile_json()['kernels']
        tot = sum(v['total_ms'] for v in pj.values())
        if best is None or tot < best[0]:
            best = (tot, pj)
    tot, pj = best
    ks = ' '.join(f"{k}={v['total_ms']:.2f}" for k, v in pj.items() if v['launches'])
    print(f"[{tag}] {nc}x{n}: total {tot:.2f} ms | {ks}", flush=True)
