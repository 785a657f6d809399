"""T2: the C++ restatement of scipy's CG (csrc/cg.cpp), fed the reference's
objective values, must reproduce scipy's iterates, evaluation count and stop
status bit for bit.  CPU only: no kernel is launched."""
import numpy as np
import pytest

from conftest import load_golden, ragged_cell
from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib


def drive(x0, objective):
    cg = _lib.CG(x0)
    requested = []
    while True:
        x = cg.step()
        if x is None:
            break
        requested.append(x)
        f, g = objective(x, len(requested) - 1)
        cg.feed(f, g)
    return requested, cg.result()


def test_golden_traces_bitwise():
    d = load_golden('cg.npz')
    for c in range(len(d['offs']) - 1):
        a, b = d['trace_offs'][c], d['trace_offs'][c + 1]
        tx, tf, tg = d['trace_x'][a:b], d['trace_f'][a:b], d['trace_g'][a:b]

        def objective(x, k):
            assert k < len(tf), (c, k)
            assert np.array_equal(x, tx[k]), (c, k, x, tx[k])
            return tf[k], tg[k]
        req, res = drive(d['x0'], objective)
        assert len(req) == b - a, c
        assert np.array_equal(res['x'], d['res_x'][c]), c
        assert res['nit'] == d['res_nit'][c], c
        assert res['nfev'] == d['res_nfev'][c], c
        assert res['status'] == d['res_status'][c], c


@pytest.mark.parametrize('seed', range(24))
def test_live_scipy_equivalence(seed):
    """Random synthetic cells: scipy.optimize.minimize on the oracle vs the
    restatement fed the same oracle."""
    from optimalinterpolation_amd import synthetic
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 90))
    x, y = synthetic.cell_obs(rng, 4e6, 4e6, n)
    mX = np.ones(n) * 0.28
    trace = []
    res = O.fit_hypers(x, y, mX, trace=trace)

    def objective(h, k):
        f, g = O.neg_log_ml(h, x, y, mX)
        return float(np.asarray(f).item()) if np.ndim(f) else float(f), g
    req, mine = drive(np.array(O.X0_PRODUCTION), objective)
    assert len(req) == len(trace)
    for k, (h, _, _) in enumerate(trace):
        assert np.array_equal(req[k], h), k
    assert np.array_equal(mine['x'], res.x)
    assert mine['nit'] == res.nit and mine['nfev'] == res.nfev and mine['status'] == res.status


def test_inf_objective_paths():
    """Objective = +inf away from a region (the reference's non-PD branch,
    GPR:139-140) must drive the line searches exactly like scipy."""
    import scipy.optimize

    def fun(h):
        if np.abs(h).max() > 3.0:
            return np.inf, np.ones(6) * np.inf
        f = float(np.sum((h - np.array([1, -2, 0.5, 2.9, -1, 0])) ** 2 * np.arange(1, 7)))
        return f, 2 * (h - np.array([1, -2, 0.5, 2.9, -1, 0])) * np.arange(1, 7)
    calls = []

    def rec(h):
        out = fun(h)
        calls.append(np.array(h).copy())
        return out
    res = scipy.optimize.minimize(rec, x0=np.zeros(6), method='CG', jac=True)
    req, mine = drive(np.zeros(6), lambda h, k: fun(h))
    assert len(req) == len(calls)
    for a, b in zip(req, calls):
        assert np.array_equal(a, b)
    assert np.array_equal(mine['x'], res.x) and mine['status'] == res.status


def _scipy_vs_restatement(fun, x0):
    import scipy.optimize
    calls = []

    def rec(h):
        calls.append(np.array(h).copy())
        return fun(h)
    with np.errstate(all='ignore'):
        res = scipy.optimize.minimize(rec, x0=x0, method='CG', jac=True)
    req, mine = drive(np.array(x0, float), lambda h, k: fun(h))
    assert len(req) == len(calls)
    for a, b in zip(req, calls):
        assert np.array_equal(a, b)
    assert np.array_equal(mine['x'], res.x, equal_nan=True)
    assert mine['status'] == res.status and mine['nit'] == res.nit and mine['nfev'] == res.nfev
    return res


@pytest.mark.parametrize('radius', [3.0, 1.5, 0.2])
def test_nan_objective_paths(radius):
    """Objective = NaN (nlZ and gradient) beyond a radius: the reference's value
    where exp over- / underflows at a trial point makes K inf / NaN and numpy's
    cholesky propagates it (GPR:120-126; the GPU path returns the same class,
    tests/test_gpu_parity.py::test_extreme_hypers_match_reference_class) --
    scipy's CG then stops with status 3 ("NaN result encountered") or backs
    off; the restatement must follow it step for step."""
    c = np.array([1, -2, 0.5, 2.9, -1, 0])

    def fun(h):
        if np.abs(h).max() > radius:
            return np.nan, np.full(6, np.nan)
        return float(np.sum((h - c) ** 2 * np.arange(1, 7))), 2 * (h - c) * np.arange(1, 7)
    _scipy_vs_restatement(fun, np.zeros(6))


def test_nan_objective_at_x0():
    """A NaN objective at the starting point (every entry of x0 overflowing):
    scipy's outcome, exactly."""
    _scipy_vs_restatement(lambda h: (np.nan, np.full(6, np.nan)), np.zeros(6))
