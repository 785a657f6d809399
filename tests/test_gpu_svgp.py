"""GPU parity of the SVGP variant (dev/sparseGP_example.ipynb
code cell 5, "NB2") through the C ABI ``oi_svgp_batch``.

Oracle: oracle/svgp_oracle.py -- a NumPy restatement of GPflow's SVGP ELBO with
a hand-derived gradient (itself checked against finite differences and torch
autograd in tests/test_svgp_oracle.py) and TF2's Adam, over the same
deterministic minibatch stream.  Parity vs GPflow itself is unpinned
(TensorFlow / GPflow absent).  The whole Adam trajectory is compared:
  parameters   |gpu - ref| <= TOL * max(1, |ref|)   (observed <= 5e-12 at 200
               steps, 1e-13 at the notebook's n = 4600, M = 50, B = 100)
  ELBO log     relative 1e-12;  predict_f mean / variance  1e-10
"""
import os

import numpy as np
import pytest

from oracle import svgp_oracle as O
from optimalinterpolation_amd import _lib, svgp

pytestmark = pytest.mark.gpu


def _cell(rng, n):
    x = np.stack([rng.uniform(-3e5, 3e5, n), rng.uniform(-3e5, 3e5, n),
                  rng.integers(0, 9, n).astype(float)], 1)
    y = 0.3 + 0.05 * np.sin(x[:, 0] / 1e5) + 0.02 * np.cos(x[:, 1] / 7e4) + rng.normal(0, 0.02, n)
    return x, y


INIT = [25e3, 25e3, 1.0, 1.0, 0.1, 0.3]  # NB2: lengthscales, kernel var, noise var .1, mean


def _run_both(x, y, M, B, iters, seed=7, log_every=10):
    Z = O.notebook_Z(x, M)
    xs = np.array([[1e4, -2e4, 4.0]])
    pred, st, params, elbo = _lib.svgp_batch(x, y, [0, len(y)], Z[None], [INIT], xs, batch=B,
                                             iterations=iters, log_every=log_every, seed=seed,
                                             want_params=True)
    p, log = O.train(x, y, Z, INIT[:3], INIT[3], INIT[4], INIT[5], B=B, iterations=iters, seed=seed,
                     log_every=log_every)
    m, v = O.predict_f(p, xs)
    return (pred[0], st[0], params[0], elbo[0] if elbo is not None else None), (m[0], v[0], p.flat(), log)


@pytest.mark.parametrize('n,M,B,iters,tol', [(300, 12, 40, 15, 1e-12), (500, 20, 64, 200, 1e-9),
                                             (30, 8, 100, 50, 1e-10), (200, 1, 16, 30, 1e-10)])
def test_trajectory_vs_oracle(n, M, B, iters, tol):
    rng = np.random.default_rng(n + M)
    x, y = _cell(rng, n)
    (pred, st, th, elbo), (m, v, th_ref, log) = _run_both(x, y, M, B, iters)
    assert st == 0
    d = np.abs(th - th_ref) / np.maximum(1.0, np.abs(th_ref))
    print(n, M, B, iters, 'param rel', d.max(), 'elbo rel', np.max(np.abs(elbo - log) / np.abs(log)))
    assert d.max() <= tol
    assert np.allclose(elbo, log, rtol=1e-12, atol=0)
    assert abs(pred[0] - m) <= 1e-10 * max(1, abs(m)) and abs(pred[1] - v) <= 1e-10 * max(1, abs(v))


def test_notebook_shape_vs_oracle():
    """NB2's configuration: n ~ 4600 observations, M = 50 (linspace Z), B = 100;
    1000 of the notebook's 10 000 Adam steps (the oracle's cost bound)."""
    rng = np.random.default_rng(46)
    x, y = _cell(rng, 4600)
    (pred, st, th, elbo), (m, v, th_ref, log) = _run_both(x, y, 50, 100, 1000)
    d = np.abs(th - th_ref) / np.maximum(1.0, np.abs(th_ref))
    print('param rel', d.max(), 'pred', pred, m, v)
    assert st == 0 and d.max() <= 1e-9
    assert np.allclose(elbo, log, rtol=1e-12, atol=0)
    assert abs(pred[0] - m) <= 1e-10 and abs(pred[1] - v) <= 1e-10 * abs(v)


def test_batch_equals_single_and_panel_modes(monkeypatch):
    """Cells of one launch are independent (cell c keyed by seed + c), and the
    LDS-resident and global-scratch panel layouts give bitwise equal results."""
    rng = np.random.default_rng(9)
    cells = [_cell(rng, n) for n in (400, 250, 333)]
    X = np.concatenate([c[0] for c in cells])
    Y = np.concatenate([c[1] for c in cells])
    offs = np.cumsum([0] + [len(c[1]) for c in cells])
    Z = np.stack([O.notebook_Z(c[0], 16) for c in cells])
    xs = np.tile([[0.0, 0.0, 4.0]], (3, 1))
    init = np.tile(INIT, (3, 1))
    pb, sb, thb, eb = _lib.svgp_batch(X, Y, offs, Z, init, xs, batch=50, iterations=60, seed=3,
                                      want_params=True)
    for c in range(3):
        p1, s1, th1, e1 = _lib.svgp_batch(cells[c][0], cells[c][1], [0, len(cells[c][1])], Z[c:c + 1],
                                          init[:1], xs[:1], batch=50, iterations=60, seed=3 + c,
                                          want_params=True)
        assert np.array_equal(p1[0], pb[c]) and np.array_equal(th1[0], thb[c]) and np.array_equal(e1[0], eb[c])
    monkeypatch.setenv('OI_SVGP_PANELS', '0')
    pg, sg, thg, eg = _lib.svgp_batch(X, Y, offs, Z, init, xs, batch=50, iterations=60, seed=3,
                                      want_params=True)
    assert np.array_equal(pg, pb) and np.array_equal(thg, thb) and np.array_equal(eg, eb)


def test_notebook_surface():
    """svgp.SVGP mirrors NB2's SVGP(x, y, xs, Z, lengthscales, kernel_variance,
    noise_variance, mean, batchsize, iterations) call and return shapes."""
    rng = np.random.default_rng(2)
    x, y = _cell(rng, 600)
    Z = svgp.notebook_Z(x, 20)
    m, v, model = svgp.SVGP(x, y, np.array([[0.0, 0.0, 4.0]]), Z, lengthscales=[25e3, 25e3, 1],
                            kernel_variance=1, noise_variance=.1, mean=0.3, batchsize=100,
                            iterations=300)
    assert m.shape == (1, 1) and v.shape == (1, 1) and v[0, 0] > 0
    assert model['Z'].shape == (20, 3) and len(model['elbo_log']) == 30
    assert model['elbo_log'][-3:].mean() > model['elbo_log'][:3].mean()
