"""Short workload for PMC passes: one SMLII round over 256 cells of n = 3000."""
import sys
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic
cells = synthetic.make_cells([3000] * 256, seed=3)
h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (256, 1))
mX = np.full(len(cells.z), cells.mean)
for _ in range(2):
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
print("ok")
