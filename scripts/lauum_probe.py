"""Time one SMLII round's k_lauum_grad on fixed cells (for epilogue-cost A/B builds)."""
import sys
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic
for n, nc in [(1600, 800), (3000, 256)]:
    cells = synthetic.make_cells([n] * nc, seed=3)
    h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
    mX = np.full(len(cells.z), cells.mean)
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
    _lib.profile_reset()
    for _ in range(3):
        _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True)
    k = _lib.profile_json()['kernels']
    print(n, nc, {a: round(b['total_ms'] / 3, 3) for a, b in k.items() if b['launches']}, flush=True)
