import sys, time
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic
for n, nc in [(500, 1000), (3000, 256)]:
    cells = synthetic.make_cells([n] * nc, seed=3)
    h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
    mX = np.full(len(cells.z), cells.mean)
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
    _lib.profile_reset()
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True)
    pj = _lib.profile_json()
    T = (n + 63) // 64
    print(f"== n={n} cells={nc} T={T}")
    for k, j, c, ms in pj['last_round']:
        extra = ''
        if k == 'k_chol_panel':
            # useful tile products in this launch: (T-1-j)*(j+1) trsm + sum_jj (j-jj+1) trtri + diag j+1 (j+1)
            tp = (T - 1 - j) * (j + 1) + sum(j - jj for jj in range(j)) + (j + 1 if j + 1 < T else 0)
            extra = f" useful {tp * 2 * 64**3 * c / ms / 1e9:6.1f} TF"
        print(f"  {k:14s} j={j:3d} cells={c:5d} {ms:8.3f} ms{extra}")
