"""Reference-shaped surface of the notebook's Nystrom variant.

Mirrors ``GP_example.ipynb`` code cell 1 (abbreviated NB1) -- the rank-M
Nystrom approximation of the per-cell GP (Williams & Seeger 2001) that the
notebook's "Approximate matrix inverse using Nystrom method" section (code
cell 5) fits and predicts with:

* ``SMLII(hypers, x, y, approx=False, M=None)``   -- NB1 SMLII, 5 log-hypers,
  ``y`` already the residual ``outputs - mX``; same return shapes
  (nlZ (1,), dnlZ (5,)), +inf on LinAlgError.
* ``GPR(x, y, xs, ell, sf2, sn2, mean, approx=False, M=None, returnprior=False)``
  -- NB1 GPR (fs, sd[, prior sd]); ``M=None`` means ``int(n/5)`` as in NB1.
* ``fit(x, y, M, x0=None)`` / ``fit_batch`` -- ``scipy.optimize.minimize(SMLII, x0,
  args=(x, y, True, M), method='CG', jac=True)`` (NB1 code cell 5) on the
  restated scipy CG of liboi.
* ``*_batch`` forms take ragged cells (xyt, y, offs) and run one liboi call.

The approx=True arithmetic runs on the GPU (liboi ``oi_nystrom_batch``:
hand-written batched eigensolver, blocked Cholesky and MFMA products of
csrc/oi_linalg.hip, fused HIP objective pass; no vendor BLAS / LAPACK); the
approx=False branch is the full GP of the main path (``oi_nlml_grad_batch`` /
``oi_gpr_batch``).  Only the inducing-row draw is host-side, exactly NB1's.
"""
import numpy as np

from . import _lib

# liboi options used by every call (device, stream, ...)
options = {}


def inducing_rows(n, M, seed=20):
    """NB1 Nystroem: ``np.random.seed(seed)`` then
    ``sorted(np.random.choice(range(n), M, replace=False))``.  Like the
    notebook it re-seeds numpy's global stream on every call."""
    np.random.seed(seed)
    return np.array(sorted(np.random.choice(range(n), M, replace=False)), dtype=np.int64)


def _ragged_sel(offs, Ms, seed=20):
    sizes = np.diff(np.asarray(offs, dtype=np.int64))
    Ms = np.broadcast_to(np.asarray(Ms, dtype=np.int64), sizes.shape)
    sel = [inducing_rows(int(n), int(M), seed) for n, M in zip(sizes, Ms)]
    soffs = np.zeros(len(sizes) + 1, dtype=np.int64)
    soffs[1:] = np.cumsum(Ms)
    return (np.concatenate(sel) if sel else np.zeros(0, np.int64)), soffs


def _linear(hypers):
    """NB1 SMLII: ell = [exp h0, exp h1, exp h2], sf2 = exp h3, sn2 = exp h4."""
    h = np.asarray(hypers, dtype=np.float64).reshape(-1, 5)
    return np.column_stack([np.exp(h[:, 0]), np.exp(h[:, 1]), np.exp(h[:, 2]), np.exp(h[:, 3]),
                            np.exp(h[:, 4])])


def SMLII_batch(hypers, xyt, y, offs, M):
    """NB1 SMLII(approx=True, M) for ragged cells: (nlZ [ncell], dnlZ [ncell x 5],
    status [ncell]); ``hypers`` [ncell x 5] log-hypers, ``M`` scalar or per cell."""
    sel, soffs = _ragged_sel(offs, M)
    nlz, grad, _, status = _lib.nystrom_batch(xyt, y, offs, sel, soffs, _linear(hypers),
                                              objective=True, predict=False, **options)
    return nlz, grad, status


def SMLII(hypers, x, y, approx=False, M=None):
    """NB1 SMLII: negative log marginal likelihood and its 5-gradient."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 3)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    offs = np.array([0, len(y)], dtype=np.int64)
    if approx:
        nlz, grad, status = SMLII_batch(np.asarray(hypers, float).reshape(1, 5), x, y, offs, M)
    else:  # NB1's exact branch is the main path's SMLII with mX = 0 (5 hypers + a dead 6th)
        h6 = np.append(np.asarray(hypers, dtype=np.float64)[:5], 0.0).reshape(1, 6)
        nlz, g6, status = _lib.nlml_grad_batch(x, y, np.zeros(len(y)), offs, h6, **options)
        grad = g6[:, :5]
    if status[0] != 0:
        return np.inf, np.ones(5) * np.inf
    return np.array([nlz[0]]), grad[0]


def GPR_batch(xyt, y, offs, xs, hyp, mean, M=None):
    """NB1 GPR(approx=True) for ragged cells: pred [ncell x 3] = (fs, sd, prior
    sd), status [ncell].  ``hyp`` [ncell x 5] LINEAR (ell_x, ell_y, ell_t, sf2,
    sn2); ``M`` None => int(n/5) per cell (NB1)."""
    sizes = np.diff(np.asarray(offs, dtype=np.int64))
    if M is None:
        M = np.array([int(n / 5) for n in sizes], dtype=np.int64)
    sel, soffs = _ragged_sel(offs, M)
    _, _, pred, status = _lib.nystrom_batch(xyt, y, offs, sel, soffs, hyp, xs=xs, mean=mean,
                                            objective=False, predict=True, **options)
    return pred, status


def GPR(x, y, xs, ell, sf2, sn2, mean, approx=False, M=None, returnprior=False):
    """NB1 GPR for one cell and one target: (fs, sd[, prior sd])."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 3)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xs = np.asarray(xs, dtype=np.float64).reshape(1, 3)
    offs = np.array([0, len(y)], dtype=np.int64)
    hyp = np.array([[ell[0], ell[1], ell[2], sf2, sn2]], dtype=np.float64)
    if approx:
        pred, status = GPR_batch(x, y, offs, xs, hyp, mean, M=None if M is None else [M])
        fs, sd, sp = np.array([[pred[0, 0]]]), np.array([pred[0, 1]]), pred[0, 2]
    else:  # full GP: the main path's predict with the residual outputs and mean 0
        out, status, _ = _lib.gpr_batch(x, y, offs, xs, 0.0, opt=False, hyp=hyp, **options)
        fs, sd, sp = np.array([mean + out[0, 0]]), np.array([out[0, 1]]), np.sqrt(sf2)
    if status[0] != 0:
        raise np.linalg.LinAlgError("Nystrom / Cholesky factorisation failed")
    return (fs, sd, sp) if returnprior else (fs, sd)


def default_x0(grid_res=25):
    """NB1 code cell 5: [log(grid_res*1000)] * 2 + [log 1, log 1, log .1]."""
    return np.array([np.log(grid_res * 1000), np.log(grid_res * 1000), np.log(1.), np.log(1.),
                     np.log(.1)])


def fit_predict_batch(xyt, y, offs, xs, mean, M, x0=None):
    """NB1 code cell 5 for every cell of a ragged batch in one liboi call
    (``oi_nystrom_fit_batch``): ``minimize(SMLII, x0, args=(x, y, True, M),
    method='CG', jac=True)`` per cell -- the restated scipy CG on the host, one
    GPU pass over the cells still iterating per round -- then
    ``GPR(approx=True, returnprior=True)`` at the fitted hypers.
    Returns (pred [ncell x 3] = (fs, sd, prior sd), x [ncell x 5] fitted
    log-hypers, info [ncell x 4] = (nit, status, nfev, objective evals))."""
    offs = np.asarray(offs, dtype=np.int64)
    sel, soffs = _ragged_sel(offs, M)
    x0 = default_x0() if x0 is None else np.asarray(x0, dtype=np.float64)
    out, status, info = _lib.nystrom_fit_batch(xyt, y, offs, sel, soffs, x0, xs, mean, **options)
    return out[:, :3], np.log(out[:, 3:]), info


def fit_batch(xyt, y, offs, M, x0=None):
    """The fit half of ``fit_predict_batch``: (x [ncell x 5] log-hypers, info)."""
    ncell = len(offs) - 1
    _, x, info = fit_predict_batch(xyt, y, offs, np.zeros((ncell, 3)), 0.0, M, x0=x0)
    return x, info


def fit(x, y, M, x0=None):
    """One cell of ``fit_batch``: the minimize() result as a dict (x [5], nit,
    status, nfev, nobj)."""
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    xh, info = fit_batch(x, y, np.array([0, len(y)]), M, x0=x0)
    return dict(x=xh[0], nit=int(info[0, 0]), status=int(info[0, 1]), nfev=int(info[0, 2]),
                nobj=int(info[0, 3]))
