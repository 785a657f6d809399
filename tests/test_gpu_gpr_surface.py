"""GPU checks of the reference-shaped surface (optimalinterpolation_amd/gpr.py)
against the reference-generated fixtures: SMLII (GPR:107-141) at T1
tolerance on smlii.npz; GPR3D(index, opt=False) / GPR3D_batch (GPR:143-191
with the smoothed-hyper lookup GPR:170-172) against gpr3d.npz's reference
2-tuples; GPR3D(index, opt=True) per cell equals the batched C-ABI call on
the same inputs bit for bit (the fit itself is T3-checked in test_gpu_fit.py)."""
import numpy as np
import pytest

from conftest import load_golden
from optimalinterpolation_amd import _lib, gpr
from test_gpr_surface import _install

pytestmark = pytest.mark.gpu


def test_smlii_shim_golden():
    d = load_golden('smlii.npz')
    for k in range(len(d['nlZ'])):
        a, b = int(d['offs'][k]), int(d['offs'][k + 1])
        x, y = d['x'][a:b].reshape(-1, 3), d['y'][a:b]
        nlz, g = gpr.SMLII(d['h'][k], x, y, np.ones(len(y)) * float(d['mean']))
        ref = d['nlZ'][k]
        if np.isinf(ref):
            assert np.isinf(nlz) and np.all(np.isinf(g))
            continue
        assert np.shape(nlz) == (1,) and np.shape(g) == (6,)
        assert abs(nlz[0] - ref) <= 1e-10 * max(1.0, abs(ref)), (k, nlz, ref)
        gs = np.abs(d['g'][k]) + 1.0
        assert np.all(np.abs(g - d['g'][k]) <= 1e-8 * gs), (k, g, d['g'][k])


def test_gpr3d_opt_false_golden():
    d = load_golden('gpr3d.npz')
    X = _install()
    hyp = d['hyp2']
    gpr.ellXs, gpr.sf2xs, gpr.sn2xs = hyp[:, 0:3].copy(), hyp[:, 3].copy(), hyp[:, 4].copy()
    one = [gpr.GPR3D(i, opt=False) for i in range(len(X))]
    many = gpr.GPR3D_batch(np.arange(len(X)), opt=False)
    assert [tuple(t) for t in one] == [tuple(t) for t in many]
    for i, (fs, sd) in enumerate(one):
        rfs, rsd = d['out2'][i]
        for a, b in ((fs, rfs), (sd, rsd)):
            assert (np.isnan(a) and np.isnan(b)) or abs(a - b) <= 1e-10 * max(1.0, abs(b)), (i, a, b)


def test_gpr3d_opt_true_equals_batched_call():
    d = load_golden('gpr3d.npz')
    X = _install()
    idx = [4, 7, 9, 11]
    got = [gpr.GPR3D(i) for i in idx]
    for i, t in zip(idx, got):
        a, b = int(d['offs'][i]), int(d['offs'][i + 1])
        out, _, _ = _lib.gpr_batch(d['x'][a:b], d['y'][a:b], [0, b - a], d['xs'][i:i + 1], float(d['mean']),
                                   x0=np.array(gpr.x0), opt=True)
        assert len(t) == 8
        assert np.array_equal(np.array(t, float), out[0], equal_nan=True), i
    assert len(gpr.GPR3D_batch(np.arange(len(X)))) == len(X)
