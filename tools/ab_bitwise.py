"""Bitwise A/B of two builds of liboi.so on the same inputs (a refactor that
must not change a single bit): objective + gradient at fixed hypers on cells
from n = 1 to 3000 (every tile-boundary class), predict at FIXED_HYPERS, and
full opt=True fits of a few day cells.  Usage (GPU box):
    python tools/ab_bitwise.py run OUT.npz        # with OI_LIB set as wanted
    python tools/ab_bitwise.py cmp A.npz B.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(out):
    from optimalinterpolation_amd import _lib, synthetic
    sizes = [1, 2, 40, 63, 64, 65, 128, 129, 200, 257, 333, 700, 1100, 1600, 2300, 3000]
    cells = synthetic.make_cells(sizes, seed=77)
    h = np.tile(np.array([np.log(2e5), np.log(2.5e5), np.log(7.), np.log(4e-3), np.log(1e-3), 0.]), (len(sizes), 1))
    nlz, grad, st = _lib.nlml_grad_batch(cells.xyt, cells.z, np.full(len(cells.z), cells.mean), cells.offs, h)
    hyp = np.tile(synthetic.FIXED_HYPERS, (len(sizes), 1))
    pred, pst, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
    day = synthetic.make_day(seed=0, max_cells=40)
    fit, fst, info = _lib.gpr_batch(day.xyt, day.z, day.offs, day.xs, day.mean,
                                    x0=np.array([np.log(25e3), np.log(25e3), 0, 0, 0, np.log(.1)]), opt=True, info=True)
    np.savez(out, nlz=nlz, grad=grad, st=st, pred=pred, pst=pst, fit=fit, fst=fst, info=info)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k], equal_nan=True)]
    for k in bad:
        d = np.abs(A[k].astype(float) - B[k].astype(float))
        print(f"DIFF {k}: max abs {np.nanmax(d):.3e} at {np.unravel_index(np.nanargmax(d), d.shape)}")
    print("bitwise equal" if not bad else f"{len(bad)} arrays differ", [f for f in A.files])
    return 0 if not bad else 1


if __name__ == '__main__':
    sys.exit(run(sys.argv[2]) if sys.argv[1] == 'run' else cmp(sys.argv[2], sys.argv[3]))
