"""T3: end-to-end GPR3D(opt=True) on the GPU vs the oracle.

scipy's CG stops on line-search failure in most cells, and its stopping point
is chaotic in floating-point noise (re-running the reference on permuted
observations moves fs by >1e-8 in ~23% of cells).  So the GPU fit is judged
as one more sample of that noise: per cell it must match the reference to
1e-6 or reach an nlZ inside the reference's own permutation envelope, and it
may miss the envelope no more often than a held-out permuted reference run
does (check_fleet); fleet medians and evaluation counts as below.
"""
import numpy as np
import pytest

from conftest import load_golden, ragged_cell
from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib, synthetic

pytestmark = pytest.mark.gpu


def nlz_at(hyp5, x, y, mean):
    h = np.r_[np.log(hyp5), np.log(.1)]
    f, _ = O.neg_log_ml(h, x, y, np.ones(len(y)) * mean)
    return float(np.asarray(f).item()) if np.ndim(f) else float(f)


def check_fleet(xyt, z, offs, xs, mean, nperm=4, seed=5):
    """Per cell: outputs agree with the reference to 1e-6, or the GPU fit is at
    least as good (in nlZ) as the worst of the reference's own runs on
    permuted copies of the cell's observations (its floating-point-noise
    envelope, built from the unpermuted run and nperm-1 permutations).  The
    last permutation is held out as one more sample of the reference's own
    noise and checked against the same envelope: the GPU may fall outside the
    envelope no more often than that held-out reference run does (+10 % of the
    cells).  Fleet: median fs rel-err <= 1e-8; the fraction of cells with fs
    rel-err > 1e-6 no larger than the reference-vs-permuted-reference fraction
    + 10 %; mean objective evaluations within 15 % of the reference's."""
    out, status, info = _lib.gpr_batch(xyt, z, offs, xs, mean, x0=np.array(O.X0_PRODUCTION),
                                       opt=True, info=True)
    prng = np.random.default_rng(seed)
    rel, rel_perm, bad, bad_ref, ev_gpu, ev_ref = [], [], [], [], [], []
    ncell = len(offs) - 1
    for c in range(ncell):
        a, b = offs[c], offs[c + 1]
        x, y = xyt[a:b], z[a:b]
        tr = []
        r8 = np.array(O.gp_cell(x, y, xs[c], mean, opt=True, trace=tr), float)
        ev_ref.append(len(tr))
        ev_gpu.append(info[c, 3])
        rel.append(abs(out[c, 0] - r8[0]) / abs(r8[0]))
        if np.allclose(out[c], r8, rtol=1e-6, atol=0, equal_nan=True):
            rel_perm.append(0.0)
            continue
        f_ref = nlz_at(r8[3:8], x, y, mean)
        f_env, fs_perm, f_held = f_ref, [], None
        for q in range(nperm):
            p = prng.permutation(len(y))
            rp = np.array(O.gp_cell(x[p], y[p], xs[c], mean, opt=True), float)
            fs_perm.append(abs(rp[0] - r8[0]) / abs(r8[0]))
            if q == nperm - 1:
                f_held = nlz_at(rp[3:8], x, y, mean)
            else:
                f_env = max(f_env, nlz_at(rp[3:8], x, y, mean))
        rel_perm.append(max(fs_perm))
        tol = 1e-8 * abs(f_ref) + 1e-9
        f_gpu = nlz_at(out[c, 3:8], x, y, mean)
        if f_gpu > f_env + tol:
            bad.append((c, len(y), f_gpu - f_ref, f_env - f_ref))
        if f_held > f_env + tol:
            bad_ref.append((c, len(y), f_held - f_ref, f_env - f_ref))
    rel, rel_perm = np.array(rel), np.array(rel_perm)
    assert len(bad) <= len(bad_ref) + 0.1 * ncell, (ncell, bad, bad_ref)
    assert np.median(rel) <= 1e-8, np.median(rel)
    assert np.mean(rel > 1e-6) <= np.mean(rel_perm > 1e-6) + 0.1, (np.mean(rel > 1e-6), np.mean(rel_perm > 1e-6))
    assert abs(np.mean(ev_gpu) / np.mean(ev_ref) - 1) <= 0.15, (np.mean(ev_gpu), np.mean(ev_ref))
    return out, info


def test_golden_gpr3d_fits():
    d = load_golden('gpr3d.npz')
    check_fleet(d['x'], d['y'], d['offs'], d['xs'], float(d['mean']))


def test_synthetic_fleet_fits():
    rng = np.random.default_rng(77)
    sizes = rng.integers(20, 260, 40)
    cells = synthetic.make_cells(sizes, seed=78)
    check_fleet(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean)
