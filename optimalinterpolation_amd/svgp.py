"""Reference-shaped surface of the dev notebook's sparse variational GP
(second half).

Mirrors ``dev/sparseGP_example.ipynb`` code cell 5 (abbreviated NB2):
``SVGP(x, y, xs, Z, lengthscales=1, kernel_variance=1, noise_variance=None,
mean=0, batchsize=None, iterations=10000)`` -- a GPflow SVGP (Matern32,
Gaussian likelihood, Constant mean, whitened) trained by TF2 Adam on
minibatches, returning ``predict_f(xs)``.  Here the whole training of every
cell runs on the GPU in one liboi call (``oi_svgp_batch``: one workgroup per
cell, all iterations in one launch).  Differences from the notebook, by
necessity: the minibatch stream is a deterministic keyed permutation (TF's
shuffle RNG cannot be reproduced), and instead of a GPflow model object the
final parameters come back as a dict.
"""
import numpy as np

from . import _lib

options = {}


def notebook_Z(x, M=50):
    """NB2: Z[:, d] = np.linspace(min x[:, d], max x[:, d], 50)."""
    x = np.asarray(x, dtype=np.float64)
    return np.stack([np.linspace(np.min(x[:, d]), np.max(x[:, d]), M) for d in range(3)], 1)


def unpack(theta, M):
    """Unconstrained parameter vector -> constrained GPflow-style values."""
    sp = lambda v: np.logaddexp(0.0, v)
    S = np.zeros((M, M))
    S[np.tril_indices(M)] = theta[6 + 4 * M:]
    return dict(lengthscales=sp(theta[:3]), kernel_variance=float(sp(theta[3])),
                noise_variance=float(sp(theta[4])) + 1e-6, mean=float(theta[5]),
                Z=theta[6:6 + 3 * M].reshape(M, 3), q_mu=theta[6 + 3 * M:6 + 4 * M], q_sqrt=S)


def SVGP_batch(xyt, y, offs, xs, Z, lengthscales, kernel_variance, noise_variance, mean,
               batchsize=100, iterations=10000, log_every=10, seed=0):
    """NB2 SVGP for every cell of a ragged batch in one GPU launch.  ``Z`` is
    [ncell x M x 3] (or one M x 3 array for all cells); the hyper arguments are
    scalars / 3-vectors or per-cell arrays.  Returns (mean [ncell], var
    [ncell], params list of dicts, elbo [ncell x nlog], status)."""
    offs = np.asarray(offs, dtype=np.int64)
    ncell = len(offs) - 1
    Z = np.asarray(Z, dtype=np.float64)
    if Z.ndim == 2:
        Z = np.broadcast_to(Z, (ncell,) + Z.shape)
    init = np.zeros((ncell, 6))
    init[:, :3] = np.broadcast_to(np.asarray(lengthscales, dtype=np.float64), (ncell, 3))
    init[:, 3] = kernel_variance
    init[:, 4] = noise_variance
    init[:, 5] = mean
    pred, status, params, elbo = _lib.svgp_batch(xyt, y, offs, Z, init, xs, batch=batchsize,
                                                 iterations=iterations, log_every=log_every,
                                                 seed=seed, want_params=True, **options)
    M = Z.shape[1]
    return pred[:, 0], pred[:, 1], [unpack(p, M) for p in params], elbo, status


def SVGP(x, y, xs, Z, lengthscales=1, kernel_variance=1, noise_variance=None, mean=0,
         batchsize=None, iterations=10000, seed=0):
    """NB2 SVGP for one cell: (mean [1,1], var [1,1], params dict).  As in the
    notebook, noise_variance None means 0.1 * var(y) and batchsize None means n."""
    x = np.asarray(x, dtype=np.float64).reshape(-1, 3)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if noise_variance is None:
        noise_variance = 0.1 * np.var(y)
    if batchsize is None:
        batchsize = len(y)
    ls = np.broadcast_to(np.asarray(lengthscales, dtype=np.float64), (3,))
    m, v, params, elbo, status = SVGP_batch(x, y, [0, len(y)], np.asarray(xs).reshape(1, 3), Z, ls,
                                            kernel_variance, noise_variance, mean,
                                            batchsize=batchsize, iterations=iterations, seed=seed)
    params[0]['elbo_log'] = elbo[0] if elbo is not None else None
    return np.array([[m[0]]]), np.array([[v[0]]]), params[0]
