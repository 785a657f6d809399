"""T3 at config-3 sizes: the GPU's GPR3D(opt=True) fit of
cells with n = 500 .. 3000 observations against the REFERENCE's own fits
(tests/golden/fit_large.npz, made by tests/golden/make_fit_large.py running
GPR_CS2S3.py:143-191 in the build container on the original observation
order and on 4 permutations of it).

scipy's CG stops on line-search failure and its stopping point moves with
rounding noise, so per cell the GPU fit must either reproduce the
reference's outputs to 1e-6 or reach an nlZ no worse than the worst of the
reference's own runs 0-3 (its permutation envelope); run 4 is a held-out
reference sample judged by the same rule, and the GPU may miss the envelope
no more often than it does (+10 % of the cells).  The optimiser's work must
match too: per n bucket the GPU's mean SMLII evaluations per cell are within
10 % of the reference's mean over its 5 runs (or inside the range the
reference's own runs span)."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib

pytestmark = pytest.mark.gpu


def nlz_at(hyp5, x, y, mean):
    """The reference's objective (oracle, bit-identical to SMLII GPR:107-141) at
    linear hypers, on the original observation order."""
    f, _ = O.neg_log_ml(np.r_[np.log(hyp5), np.log(.1)], x, y, np.ones(len(y)) * mean)
    return float(np.asarray(f).item()) if np.ndim(f) else float(f)


def test_config3_size_fits_against_reference():
    d = load_golden('fit_large.npz')
    x, y, offs, xs, mean = d['x'].reshape(-1, 3), d['y'], d['offs'], d['xs'], float(d['mean'])
    out8, evals, nlz, sizes = d['out8'], d['evals'], d['nlz'], d['sizes']
    ncell = len(sizes)
    out, status, info = _lib.gpr_batch(x, y, offs, xs, mean, x0=np.array(O.X0_PRODUCTION), opt=True,
                                       info=True)
    assert np.all(status == 0) and np.isfinite(out).all()
    bad, bad_ref, report = [], [], []
    for c in range(ncell):
        a, b = offs[c], offs[c + 1]
        ref = out8[c, 0]
        f_env = max(nlz[c, :4])
        tol = 1e-8 * abs(nlz[c, 0]) + 1e-9
        same = np.allclose(out[c], ref, rtol=1e-6, atol=0)
        f_gpu = nlz_at(out[c, 3:8], x[a:b], y[a:b], mean)
        report.append((int(sizes[c]), int(info[c, 3]), list(evals[c]), f_gpu - nlz[c, 0], f_env - nlz[c, 0]))
        if not same and f_gpu > f_env + tol:
            bad.append(report[-1])
        if nlz[c, 4] > f_env + tol:
            bad_ref.append(c)
    assert len(bad) <= len(bad_ref) + 0.1 * ncell, (bad, bad_ref, report)
    for n in np.unique(sizes):
        m = sizes == n
        g = float(np.mean(info[m, 3]))
        r = float(np.mean(evals[m]))
        lo, hi = float(evals[m].min()), float(evals[m].max())
        assert abs(g / r - 1) <= 0.10 or lo <= g <= hi, (int(n), g, r, lo, hi, report)
