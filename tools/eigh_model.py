"""NumPy model of the hand-written batched eigensolver (csrc/oi_linalg.hip)
used by the Nystrom variant in place of LAPACK/rocSOLVER syevd
(GP_example.ipynb's ``np.linalg.eigh(Kmm)``): the same algorithm step for
step, so its accuracy can be checked against numpy on the CPU before the
kernels run.

  1. blocked Householder tridiagonalisation (LAPACK dsytrd / dlatrd, lower):
     panels of NBT columns, per column the symv with the panel's corrections,
     rank-2 NBT trailing update per panel; V (unit lower) and T (dlarft,
     forward columnwise) kept per panel for the back-transform;
  2. eigenvalues of the tridiagonal by bisection on Sturm counts (dstebz);
  3. eigenvectors of the tridiagonal by inverse iteration with partial
     pivoting (dlagtf / dlagts), a pseudo-random start per eigenvalue;
  4. block classical Gram-Schmidt twice (BCGS2) over blocks of 128 and
     panels of 32 vectors,
     Cholesky QR twice inside a panel; where a column collapses (numerically
     repeated eigenvalues) Gram-Schmidt column by column with a fresh start
     vector;
  5. back-transform U = Q Z, one block reflector I - V T V' per panel.
"""
import numpy as np

NBT = 32


def sytrd(A0, nbt=NBT):
    A = np.array(A0, dtype=float)
    M = A.shape[0]
    d, e, tau = np.zeros(M), np.zeros(max(M - 1, 0)), np.zeros(max(M - 1, 0))
    panels = []
    p = 0
    while p < M - 1:
        nb = min(nbt, M - 1 - p)
        V = np.zeros((M, nb))
        W = np.zeros((M, nb))
        for i in range(nb):
            g = p + i
            # (1) bring column g up to date with the panel so far (rows g..M-1)
            if i > 0:
                A[g:, g] -= V[g:, :i] @ W[g, :i] + W[g:, :i] @ V[g, :i]
            # (2) reflector annihilating A(g+2:, g)
            alpha = A[g + 1, g]
            xn = np.sqrt(np.sum(A[g + 2:, g] ** 2))
            if xn == 0.0:
                t, beta = 0.0, alpha
                v = np.zeros(M)
                v[g + 1] = 1.0
            else:
                beta = -np.copysign(np.hypot(alpha, xn), alpha)
                t = (beta - alpha) / beta
                v = np.zeros(M)
                v[g + 1] = 1.0
                v[g + 2:] = A[g + 2:, g] / (alpha - beta)
            e[g], tau[g] = beta, t
            d[g] = A[g, g]
            # (3) w = tau (A22 v - V (W'v) - W (V'v)); w += -tau/2 (w'v) v
            L = np.tril(A[g + 1:, g + 1:])
            A22 = L + np.tril(L, -1).T
            y = A22 @ v[g + 1:]
            wv_, vv_ = W[g + 1:, :i].T @ v[g + 1:], V[g + 1:, :i].T @ v[g + 1:]
            # w'v from the dots (round 5, k_sy_w: no reduction over w):
            # w'v = tau (y'v - 2 (W'v).(V'v))
            a2 = -0.5 * t * (t * (y @ v[g + 1:] - 2.0 * (wv_ @ vv_)))
            y -= V[g + 1:, :i] @ wv_ + W[g + 1:, :i] @ vv_
            w = np.zeros(M)
            w[g + 1:] = t * y + a2 * v[g + 1:]
            V[:, i], W[:, i] = v, w
        # trailing update (rows / columns from p + nb)
        q = p + nb
        A[q:, q:] -= V[q:] @ W[q:].T + W[q:] @ V[q:].T
        # T of the block reflector: H_p ... H_{p+nb-1} = I - V T V'
        T = np.zeros((nb, nb))
        for i in range(nb):
            T[i, i] = tau[p + i]
            if i:
                T[:i, i] = -tau[p + i] * (T[:i, :i] @ (V[:, :i].T @ V[:, i]))
        panels.append((p, V, T))
        p = q
    d[M - 1] = A[M - 1, M - 1]
    return d, e, panels


def sturm_count(d, e2, x, pivmin):
    c, q = 0, d[0] - x
    if abs(q) < pivmin:
        q = -pivmin
    c += q < 0
    for i in range(1, len(d)):
        q = d[i] - x - e2[i - 1] / q
        if abs(q) < pivmin:
            q = -pivmin
        c += q < 0
    return c


def stebz(d, e):
    M = len(d)
    e2 = e ** 2
    ae = np.abs(np.r_[0.0, e]) + np.abs(np.r_[e, 0.0])
    gl, gu = np.min(d - ae), np.max(d + ae)
    tnorm = max(abs(gl), abs(gu))
    pivmin = np.finfo(float).tiny * max(1.0, np.max(e2) if M > 1 else 1.0)
    gl -= 2.1 * tnorm * np.finfo(float).eps * M + 2.1 * pivmin
    gu += 2.1 * tnorm * np.finfo(float).eps * M + 2.1 * pivmin
    lam = np.zeros(M)
    eps = np.finfo(float).eps
    for k in range(M):       # eigenvalue k (0-based): count(x) <= k  <=>  x <= lambda_k
        lo, hi = gl, gu
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if hi - lo <= 2 * eps * max(abs(lo), abs(hi)) + pivmin or mid == lo or mid == hi:
                break
            if sturm_count(d, e2, mid, pivmin) <= k:
                lo = mid
            else:
                hi = mid
        lam[k] = 0.5 * (lo + hi)
    return lam, tnorm


def start_vector(k, M):
    i = np.arange(M, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B97F4A7C15) + np.uint64(k + 1) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(
        0xFFFFFFFFFFFFFFFF)
    h ^= h >> np.uint64(31)
    h = (h * np.uint64(0x94D049BB133111EB)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    h ^= h >> np.uint64(29)
    return (h >> np.uint64(11)).astype(float) / 2.0 ** 53 * 2.0 - 1.0


def lagtf(d, e, lam):
    """T - lam I = P L U (dlagtf): a diag of U, b first / c second superdiagonal, l multipliers, piv."""
    M = len(d)
    a = d - lam
    b = np.r_[e, 0.0].copy()
    c = np.zeros(M)
    l = np.zeros(M)
    piv = np.zeros(M, dtype=bool)
    sub = np.r_[e, 0.0]
    for k in range(M - 1):
        if abs(a[k]) >= abs(sub[k]):
            m = sub[k] / a[k] if a[k] != 0.0 else 0.0
            l[k] = m
            a[k + 1] -= m * b[k]
        else:
            m = a[k] / sub[k]
            l[k] = m
            piv[k] = True
            a[k] = sub[k]
            t = a[k + 1]
            a[k + 1] = b[k] - m * t
            if k < M - 2:
                c[k] = b[k + 1]
                b[k + 1] = -m * c[k]
            b[k] = t
    return a, b, c, l, piv


def lagts(a, b, c, l, piv, y, tol):
    M = len(a)
    y = y.copy()
    for k in range(M - 1):
        if piv[k]:
            y[k], y[k + 1] = y[k + 1], y[k] - l[k] * y[k + 1]
        else:
            y[k + 1] -= l[k] * y[k]
    for k in range(M - 1, -1, -1):
        t = y[k]
        if k < M - 1:
            t -= b[k] * y[k + 1]
        if k < M - 2:
            t -= c[k] * y[k + 2]
        ak = a[k]
        if abs(ak) < tol:
            ak = tol if ak >= 0 else -tol
        y[k] = t / ak
    return y


def stein(d, e, lam, tnorm, iters=2):
    M = len(d)
    Z = np.zeros((M, M))
    eps = np.finfo(float).eps
    tol = eps * tnorm
    for k in range(M):
        a, b, c, l, piv = lagtf(d, e, lam[k])
        x = start_vector(k, M)
        for _ in range(iters):
            x = lagts(a, b, c, l, piv, x, tol)
            x /= np.max(np.abs(x))
        Z[:, k] = x / np.linalg.norm(x)
    return Z


def mgs(Z, p, q):
    M = Z.shape[0]
    for j in range(p, q):
        for tries in range(3):
            n0 = np.linalg.norm(Z[:, j])
            for _ in range(2):
                Z[:, j] -= Z[:, p:j] @ (Z[:, p:j].T @ Z[:, j])
            n1 = np.linalg.norm(Z[:, j])
            if n1 > 1e-2 * n0:
                break
            x = start_vector(j + 7919 * (tries + 1), M)
            for _ in range(2):
                x -= Z[:, :j] @ (Z[:, :j].T @ x)
            Z[:, j] = x
        Z[:, j] /= np.linalg.norm(Z[:, j])


def cholqr2(Z, p, q):
    """Z[:, p:q] <- Q of its QR, twice (k_orth_panel); False on a collapse
    (a pivot keeping <= 1e-4 of its column's squared norm), Z then unchanged
    by the failing pass."""
    for _ in range(2):
        G = Z[:, p:q].T @ Z[:, p:q]
        R = np.triu(G).copy()
        nb = q - p
        for j in range(nb):
            if not R[j, j] > 1e-4 * G[j, j]:
                return False
            R[j, j] = np.sqrt(R[j, j])
            R[j, j + 1:] /= R[j, j]
            R[j + 1:, j + 1:] -= np.triu(np.outer(R[j, j + 1:], R[j, j + 1:]))
        Z[:, p:q] = Z[:, p:q] @ np.linalg.inv(R)
    return True


def bcgs2(Z, nb=32, ob=128):
    """Two-level BCGS2 (round 5, OI_ORTH_BLOCK = ob): each ob-column block
    projected out of every earlier block twice, then BCGS2 between its
    nb-column panels; ob = nb is plain panel-wise BCGS2."""
    M, K = Z.shape
    Z = Z.copy()

    def project(lo, p, q):
        for _ in range(2):
            H = Z[:, lo:p].T @ Z[:, p:q]
            Z[:, p:q] -= Z[:, lo:p] @ H

    for P in range(0, K, ob):
        Q = min(K, P + ob)
        if P > 0:
            project(0, P, Q)
        for p in range(P, Q, nb):
            q = min(K, p + nb)
            if p > P:
                project(P, p, q)
            if not cholqr2(Z, p, q):
                mgs(Z, p, q)
    return Z


def ormtr(panels, Z):
    U = Z.copy()
    for p, V, T in reversed(panels):
        U -= V @ (T @ (V.T @ U))
    return U


def eigh(A):
    d, e, panels = sytrd(A)
    lam, tnorm = stebz(d, e)
    Z = stein(d, e, lam, tnorm)
    # the bottom cluster (consecutive gaps <= 1e3 eps ||T||): random starts, no
    # inverse iteration; orthogonalisation in descending eigenvalue order
    eps = np.finfo(float).eps
    nb0 = 1
    while nb0 < len(lam) and lam[nb0] - lam[nb0 - 1] <= 1e3 * eps * tnorm:
        nb0 += 1
    if nb0 >= 2:
        for k in range(nb0):
            x = start_vector(k, len(lam))
            Z[:, k] = x / np.linalg.norm(x)
    Z = bcgs2(Z[:, ::-1])[:, ::-1]
    return lam, ormtr(panels, Z)


if __name__ == '__main__':
    import sys
    sys.path.insert(0, '.')
    from scipy.spatial.distance import pdist, squareform
    rng = np.random.default_rng(0)
    for M, ell, dup in ((70, 3e4, False), (160, 6e4, False), (200, 2e5, True), (300, 9e4, False),
                        (240, 4e5, True), (260, 1e6, False)):
        g = np.arange(-12, 13) * 25e3
        sites = np.array([(a, b, t) for a in g for b in g for t in range(9)])
        x = sites[rng.choice(len(sites), M, replace=False)]
        if dup:
            x[M // 2:M // 2 + 10] = x[:10]
        Q = squareform(pdist(np.sqrt(3) * x / np.array([ell, ell, 3.0])))
        A = 6e-3 * (1 + Q) * np.exp(-Q)
        lam, U = eigh(A)
        s, u = np.linalg.eigh(A)
        nrm = np.abs(s).max()
        orth = np.abs(U.T @ U - np.eye(M)).max()
        res = np.abs(A @ U - U * lam).max() / nrm
        # invariant: the clamped pseudo-inverse NB1 uses
        def pinv(ss, uu):
            ss = ss.copy()
            ss[ss <= 0] = 1e-12
            return (uu / ss) @ uu.T
        good = s > 1e-8 * nrm
        print(f"M={M} dup={dup}: eigenvalue err {np.abs(lam - s).max() / nrm:.2e}, orth {orth:.2e}, "
              f"residual {res:.2e}, cond {nrm / s[good].min():.1e}")
