"""Reference-shaped Python surface of the hot path, backed by liboi (HIP).

Mirrors ``2021_paper_production/GPR_CS2S3.py`` (``GPR:`` below):

* ``SMLII(hypers, x, y, mX)``  -- GPR:107-141, same arguments / return shapes
  (nlZ shape (1,), dnlZ (6,)), +inf on a non-PD covariance.
* ``GPR3D(index, opt=True)``   -- GPR:143-191, reads the same module globals
  (``X_tree, X, x_train, y_train, t_train, z, radius, mean, T_mid, x0,
  ellXs, sf2xs, sn2xs``) and returns the same 8-tuple / 2-tuple, NaNs on
  failure.
* ``GPR3D_batch(indices, opt=True)`` -- what the per-cell loops GPR:258-261
  and GPR:316-319 become: one call for all of a rank's cells.

All arithmetic runs on the GPU through liboi; the neighbour query (cKDTree,
GPR:159) stays on the host exactly as in the reference.
"""
import numpy as np

from . import _lib

# ---- module globals GPR3D reads (GPR:159-172); the driver assigns them ----
X_tree = None
X = None
x_train = None
y_train = None
t_train = None
z = None
radius = 300            # km (GPR:208)
mean = None             # prior mean (GPR:212)
T_mid = 4               # (GPR:207)
x0 = [np.log(25 * 1000), np.log(25 * 1000), np.log(1.), np.log(1.), np.log(1.), np.log(.1)]  # GPR:217
ellXs = None
sf2xs = None
sn2xs = None

# liboi options used by every call (device, stream, pool size, profiling ...)
options = {}


def SMLII(hypers, x, y, mX):
    """Negative log marginal likelihood and gradient of one cell (GPR:107-141)."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 3)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    mX = np.broadcast_to(np.asarray(mX, dtype=np.float64), y.shape)
    h = np.asarray(hypers, dtype=np.float64).reshape(1, 6)
    nlz, grad, status = _lib.nlml_grad_batch(x, y, mX, np.array([0, len(y)]), h, **options)
    if status[0] != 0:
        return np.inf, np.ones(6) * np.inf
    return np.array([nlz[0]]), grad[0]


def SMLII_batch(hypers, cells):
    """SMLII for many cells at once: ``cells`` is a synthetic.RaggedCells-like
    object (xyt, z, offs, mean); returns (nlZ [ncell], dnlZ [ncell x 6])."""
    mX = np.full(len(cells.z), cells.mean)
    nlz, grad, _ = _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, hypers, **options)
    return nlz, grad


def _neighbours(indices):
    """GPR:159-164 for a list of cell indices -> ragged arrays."""
    ids = [X_tree.query_ball_point(x=X[i, :], r=radius * 1000) for i in indices]
    offs = np.zeros(len(indices) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(i) for i in ids])
    cat = np.concatenate([np.asarray(i, dtype=np.int64) for i in ids]) if ids else np.zeros(0, np.int64)
    xyt = np.stack([x_train[cat], y_train[cat], t_train[cat]], axis=1) if len(cat) else np.zeros((0, 3))
    xs = np.stack([X[indices, 0], X[indices, 1], np.full(len(indices), float(T_mid))], axis=1)
    return xyt, z[cat], offs, xs


_lookup_cache = {'key': None, 'first': None}


def _first_match_rows():
    """GPR:170 ``np.where((X[:,0]==X[index,0]) & (X[:,1]==X[index,1]))`` then
    ``[0]`` (GPR:171): for every cell the FIRST row of ``X`` with the same
    coordinates.  Built once per content of ``X`` (keyed on its bytes) instead
    of once per call, so the reference-style per-cell loop stays O(ncell)."""
    Xa = np.ascontiguousarray(X, dtype=np.float64)
    key = (Xa.shape, hash(Xa.tobytes()))
    if _lookup_cache['key'] != key:
        # rows sorted by (x, y) with ties by index: a group's first row is its first match
        order = np.lexsort((np.arange(len(Xa)), Xa[:, 1], Xa[:, 0]))
        xs, ys = Xa[order, 0], Xa[order, 1]
        new = np.ones(len(order), dtype=bool)
        new[1:] = (xs[1:] != xs[:-1]) | (ys[1:] != ys[:-1])
        grp = np.cumsum(new) - 1
        first = np.empty(len(Xa), dtype=np.int64)
        first[order] = order[new][grp]
        _lookup_cache.update(key=key, first=first)
    return _lookup_cache['first']


def _smoothed_hypers(indices):
    """GPR:170-172: hyper lookup by exact coordinate match (first match)."""
    rows = _first_match_rows()[np.asarray(indices, dtype=np.int64)]
    return np.column_stack([ellXs[rows, 0], ellXs[rows, 1], ellXs[rows, 2], sf2xs[rows], sn2xs[rows]])


def GPR3D_batch(indices, opt=True):
    """GPR3D for every index in one batched GPU call; returns a list of tuples."""
    indices = np.asarray(indices, dtype=np.int64).reshape(-1)
    if len(indices) == 0:
        return []
    xyt, zz, offs, xs = _neighbours(indices)
    if opt:
        out, status, _ = _lib.gpr_batch(xyt, zz, offs, xs, mean, x0=np.asarray(x0, float)[:6],
                                        opt=True, **options)
        return [tuple(np.float64(v) for v in row) for row in out]
    out, status, _ = _lib.gpr_batch(xyt, zz, offs, xs, mean, opt=False,
                                    hyp=_smoothed_hypers(indices), **options)
    return [(np.float64(row[0]), np.float64(row[1])) for row in out]


def GPR3D(index, opt=True):
    """Gaussian Process Regression for one grid cell (GPR:143-191)."""
    return GPR3D_batch([index], opt=opt)[0]


def gpr_cells(cells, opt=True, x0=None, hyp=None, info=False, **kw):
    """Lower-level batched entry on a RaggedCells object (xyt, z, offs, xs, mean)."""
    o = dict(options)
    o.update(kw)
    if x0 is None:
        x0 = globals()['x0']
    return _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean,
                          x0=np.asarray(x0, float)[:6] if opt else None, opt=opt,
                          hyp=hyp, info=info, **o)
