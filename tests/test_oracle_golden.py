"""The CPU oracle (oracle/gp_oracle.py) against fixtures made by running the
reference itself (tests/golden/make_golden.py).  Same machine, same NumPy ->
bit-identical results are required."""
import numpy as np
import pytest

from conftest import load_golden, ragged_cell
from oracle import gp_oracle as O

# bitwise against fixtures made at OpenBLAS's default thread count (conftest)
pytestmark = pytest.mark.blas_default


def _same(a, b):
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


def test_smlii_bitwise():
    d = load_golden('smlii.npz')
    for k in range(len(d['nlZ'])):
        x, y = ragged_cell(d, k)
        f, g = O.neg_log_ml(d['h'][k], x, y, np.ones(len(y)) * float(d['mean']))
        f = float(np.asarray(f).item()) if np.ndim(f) else float(f)
        assert f == d['nlZ'][k] or (np.isnan(f) and np.isnan(d['nlZ'][k])), k
        assert _same(g, d['g'][k]), k


def test_cg_trace_bitwise():
    d = load_golden('cg.npz')
    ncell = len(d['offs']) - 1
    for c in range(ncell):
        x, y = ragged_cell(d, c)
        tr = []
        res = O.fit_hypers(x, y, np.ones(len(y)) * float(d['mean']), x0=d['x0'], trace=tr)
        a, b = d['trace_offs'][c], d['trace_offs'][c + 1]
        assert len(tr) == b - a, c
        for i, (h, f, g) in enumerate(tr):
            assert _same(h, d['trace_x'][a + i]) and f == d['trace_f'][a + i] and _same(g, d['trace_g'][a + i]), (c, i)
        assert _same(res.x, d['res_x'][c])
        assert res.nit == d['res_nit'][c] and res.nfev == d['res_nfev'][c] and res.status == d['res_status'][c]


def test_gpr3d_bitwise():
    d = load_golden('gpr3d.npz')
    for c in range(len(d['offs']) - 1):
        x, y = ragged_cell(d, c)
        out8 = O.gp_cell(x, y, d['xs'][c], float(d['mean']), opt=True, x0=O.X0_PRODUCTION)
        assert _same(out8, d['out8'][c]), c
        out2 = O.gp_cell(x, y, d['xs'][c], float(d['mean']), opt=False, hyp=d['hyp2'][c])
        assert _same(out2, d['out2'][c]), c


def test_predict64_bitwise():
    d = load_golden('predict64.npz')
    for c in range(64):
        x, y = ragged_cell(d, c)
        out2 = O.gp_cell(x, y, d['xs'][c], float(d['mean']), opt=False, hyp=d['hyp'][c])
        assert _same(out2, d['out2'][c]), c


def test_edge_n0_semantics():
    """n=0 => CG stops at x0, (mean, 1.0, -0.0, 25000, 25000, 1, 1, 1)."""
    out = O.gp_cell(np.zeros((0, 3)), np.zeros(0), [4e6, 4e6, 4.0], 0.28, opt=True)
    assert out[0] == 0.28 and out[1] == 1.0 and out[2] == 0.0 and np.signbit(out[2])
    assert np.allclose(out[3:], [25000, 25000, 1, 1, 1], rtol=0, atol=1e-9)


def test_nystrom_oracle_bitwise():
    """oracle/nystrom_oracle.py == the notebook's own Nystroem / SMLII(approx) /
    GPR(approx) (fixtures: tests/golden/make_nystrom_golden.py)."""
    from oracle import nystrom_oracle as N
    d = load_golden('nystrom.npz')
    for c in range(len(d['nlz'])):
        a, b = d['offs'][c], d['offs'][c + 1]
        x, y, h, M = d['x'][a:b], d['y'][a:b], d['h'][c], int(d['M'][c])
        f, g = N.neg_log_ml(h, x, y, M)
        assert float(np.asarray(f).item()) == d['nlz'][c], c
        assert _same(g, d['grad'][c]), c
        fs, sd, sp = N.predict(x, y, d['xs'], list(np.exp(h[:3])), np.exp(h[3]), np.exp(h[4]),
                               float(d['mean']), M)
        assert float(np.asarray(fs).item()) == d['fs'][c], c
        assert _same(np.asarray(sd).reshape(-1)[:1], d['sd'][c:c + 1]), c
        assert float(sp) == d['sprior'][c], c
