import sys
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic
cells = synthetic.make_cells([3000] * 256, seed=3)
nc = cells.ncell
h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
mX = np.full(len(cells.z), cells.mean)
_lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
_lib.profile_reset()
_lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True)
pj = _lib.profile_json()
rows = {}
for k, j, c, ms in pj['last_round']:
    rows.setdefault(j, {})[k] = ms
for j in sorted(rows):
    print(j, {k: round(v, 3) for k, v in rows[j].items()})
