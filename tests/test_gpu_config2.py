"""Config 2 at its own shape (VERDICT r4 "next" item 7): pass 2 of the
reference -- GPR3D(index, opt=False) over every cell with fixed hypers
(GPR:316-319, predict block GPR:173-182) -- as the bench's predict workload
runs it: one batch of 1 000 cells x n = 500 at synthetic.FIXED_HYPERS.

  * T1 on a stratified 32 cells (spread over the batch order): fs, sd and lZ
    within 1e-10 * max(1, |ref|) of the oracle's predict (the bit-exact
    restatement of GPR:173-182);
  * the same 1 000 cells in 8 smaller batches give bitwise the same rows
    (a cell's arithmetic never depends on its batch);
  * every cell succeeds (status 0) and its outputs are finite.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

RTOL = 1e-10


def _batch(seed=0):
    # bench.py --workload predict, step 0: make_cells([500] * 1000, seed=seed + 7919 * k + rank)
    return synthetic.make_cells([500] * 1000, seed=seed)


def test_config2_batch_t1_and_batch_independence():
    cells = _batch()
    hyp = np.tile(synthetic.FIXED_HYPERS, (cells.ncell, 1))
    out, status, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
    assert out.shape[0] == 1000 and np.all(status == 0)
    assert np.all(np.isfinite(out[:, :3]))
    pick = np.linspace(0, cells.ncell - 1, 32).round().astype(int)
    worst = 0.0
    for c in pick:
        x, y, xs = cells.cell(int(c))
        fs, sd, lz = O.predict(x, y, xs, cells.mean, hyp[c, :3], hyp[c, 3], hyp[c, 4])
        ref = np.array([fs[0], sd[0], lz])
        err = np.abs(out[c, :3] - ref) / np.maximum(1.0, np.abs(ref))
        worst = max(worst, float(err.max()))
        assert np.all(err <= RTOL), (int(c), out[c, :3], ref, err)
    print(f"config 2 T1: 32 cells, worst relative error {worst:.2e}")
    # the same cells in 8 batches of 125: bitwise the same rows
    for b in range(8):
        idx = np.arange(125 * b, 125 * (b + 1))
        sub = cells.subset(idx)
        o2, s2, _ = _lib.gpr_batch(sub.xyt, sub.z, sub.offs, sub.xs, sub.mean, opt=False, hyp=hyp[idx])
        assert np.array_equal(o2, out[idx], equal_nan=True), b
        assert np.array_equal(s2, status[idx])
