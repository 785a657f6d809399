"""CPU oracle for the Nystrom-approximated GP of the reference notebook
(GP_example.ipynb, code cell 1; abbreviated NB1) -- TEST INFRASTRUCTURE ONLY
(same rules as gp_oracle.py).

Restates, with the same NumPy operations in the same order:
* ``nystroem``   <- ``Nystroem`` (Williams & Seeger rank-M approximation of K,
                    inverted with the Woodbury identity; ``np.random.seed(20)``
                    + ``np.random.choice(range(n), M, replace=False)``, sorted)
* ``neg_log_ml`` <- ``SMLII(hypers, x, y, approx=True, M)`` (5 log-hypers; y is
                    already the residual outputs - mX, as the notebook passes it)
* ``predict``    <- ``GPR(x, y, xs, ell, sf2, sn2, mean, approx=True, M,
                    returnprior=True)``

Pinned bit-for-bit to tests/golden/nystrom.npz, which
tests/golden/make_nystrom_golden.py produced by executing the notebook's own
function definitions (tests/test_oracle_golden.py).
"""
import numpy as np
from numpy.linalg import multi_dot as mdot

from .gp_oracle import matern32


def inducing_indices(n, M, seed=20):
    """NB1 Nystroem: np.random.seed(20); sorted(np.random.choice(range(n), M,
    replace=False)) -- the legacy global RandomState stream."""
    rs = np.random.RandomState(seed)
    return np.array(sorted(rs.choice(range(n), M, replace=False)), dtype=np.int64)


def nystroem(x, y, M, ell, sf2, sn2, seed=20, opt=False):
    n = len(y)
    sel = inducing_indices(n, M, seed)
    Kmm = matern32(x[sel, :], ell, sf2)
    Knm = matern32(x, ell, sf2, xs=x[sel, :])
    Vi = np.eye(n) / sn2
    s, u = np.linalg.eigh(Kmm)
    s[s <= 0] = 1e-12
    s_tilde = n * s / M
    u_tilde = np.sqrt(M / n) * np.dot(Knm, u) / s
    L = np.linalg.cholesky(np.diag(1 / s_tilde) + mdot([u_tilde.T, Vi, u_tilde]))
    alpha = np.linalg.solve(L.T, np.linalg.solve(L, np.dot(u_tilde.T, Vi)))
    Ki = Vi - mdot([Vi, u_tilde, alpha])
    if opt:
        L_tilde = np.sqrt(s_tilde) * u_tilde
        det = np.linalg.slogdet(np.eye(M) * sn2 + np.dot(L_tilde.T, L_tilde))
        return Ki, np.atleast_2d(np.dot(Ki, y)).T, (det[0] * det[1]) / 2
    return Ki, np.atleast_2d(np.dot(Ki, y)).T


def neg_log_ml(hypers, x, y, M):
    """SMLII(..., approx=True, M): nlZ (1x1) and the 5-vector gradient; note the
    notebook's quirks kept: the exact K and dK in the gradient terms, the
    factor 2 on components 3 and 4, and a log-determinant without the
    (n - M) log sn2 term."""
    ell = [np.exp(hypers[0]), np.exp(hypers[1]), np.exp(hypers[2])]
    sf2 = np.exp(hypers[3])
    sn2 = np.exp(hypers[4])
    n = len(y)
    Kx, dK = matern32(x, ell, sf2, grad=True)
    try:
        Ki, A, det = nystroem(x, y, M=M, ell=ell, sf2=sf2, sn2=sn2, opt=True)
        nlZ = np.dot(y.T, A) / 2 + det + n * np.log(2 * np.pi) / 2
        Q = Ki - np.dot(A, A.T)
        dnlZ = np.zeros(len(hypers))
        for theta in range(len(hypers)):
            if theta < 3:
                dnlZ[theta] = (Q * dK[theta, :, :]).sum() / 2
            elif theta == 3:
                dnlZ[theta] = (Q * (2 * Kx)).sum() / 2
            elif theta == 4:
                dnlZ[theta] = sn2 * np.trace(Q)
    except np.linalg.LinAlgError:
        nlZ = np.inf
        dnlZ = np.ones(len(hypers)) * np.inf
    return nlZ, dnlZ


def predict(x, y, xs, ell, sf2, sn2, mean, M):
    """GPR(..., approx=True, M, returnprior=True): (fs, sd, prior sd)."""
    Kxsx = matern32(x, ell, sf2, xs=xs)
    Kxs = matern32(xs, ell, sf2)
    Ki, A = nystroem(x, y, M=M, ell=ell, sf2=sf2, sn2=sn2)
    err = mdot([Kxsx.T, Ki, Kxsx])
    fs = mean + np.dot(Kxsx.T, A)
    with np.errstate(invalid='ignore'):
        sfs2 = np.sqrt((Kxs - err).diagonal())
    return fs, sfs2, np.sqrt(Kxs[0][0])
