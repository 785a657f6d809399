"""CPU oracle for the dev notebook's sparse variational GP -- TEST
INFRASTRUCTURE ONLY (same rules as gp_oracle.py).

Reference: dev/sparseGP_example.ipynb code cell 5 (abbreviated NB2), function
``SVGP(x, y, xs, Z, lengthscales, kernel_variance, noise_variance, mean,
batchsize, iterations)``: a GPflow ``SVGP`` (Matern32 kernel, Gaussian
likelihood, Constant mean, ``num_data=n``) trained with ``tf.optimizers.Adam()``
on minibatches, then ``predict_f(xs)``.  TensorFlow and GPflow are NOT
installed here (the reference pins no versions; the notebook ran GPflow 2.x on
TF 2.x), so this module restates their published algorithms:

* GPflow 2 ``Matern32``: k = variance (1 + sqrt3 r) exp(-sqrt3 r),
  r = sqrt(max(r2, 1e-36)), r2 the squared distance of X / lengthscales.
* parameters and transforms: lengthscales, variance: softplus; likelihood
  variance: softplus + 1e-6; constant mean c, inducing inputs Z, q_mu:
  identity; q_sqrt: lower-triangular (FillTriangular), initialised to I;
  q_mu to 0; whiten=True; jitter 1e-6 on K_uu.
* ELBO (whitened):  sum_b E_q[log N(y_b | f_b, s2)] * n / B - KL(q(v) || N(0, I)),
  q(f_b) = N(c + A_b' q_mu, kdiag - |A_b|^2 + |S' A_b|^2),  A = L^-1 K_uf,
  L = chol(K_uu + 1e-6 I); training loss = -ELBO.
* TF2 Adam (lr 1e-3, beta1 .9, beta2 .999, eps 1e-7):
  m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
  x -= lr sqrt(1-b2^t) / (1-b1^t) * m / (sqrt(v) + eps).

Deviation (documented): tf.data's ``repeat().shuffle(n)`` stream is not
reproducible without TensorFlow's RNG; the minibatch stream here is a
deterministic per-epoch permutation (a keyed 4-round Feistel network on
integers, cycle-walked into [0, n)), batches being consecutive runs of B
stream positions.  The notebook's logging call ``training_loss()`` every 10
steps consumes one extra minibatch from the same iterator; ``log_every``
mirrors that.

The gradient is derived by hand (reverse mode through the Cholesky via
Murray's formula) and checked against finite differences and torch autograd
in tests/test_svgp_oracle.py.  **Parity unpinned** against GPflow itself.
"""
import numpy as np

SQRT3 = np.sqrt(3.0)
JITTER = 1e-6
LIK_LOWER = 1e-6
M64 = (1 << 64) - 1


# ------------------------------------------------------------ minibatches
def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(M64)
    return z ^ (z >> np.uint64(31))


def permute(i, n, seed, epoch):
    """Keyed bijection of [0, n) (vectorised over i): 4-round Feistel network on
    2h bits (4^h >= n), cycle-walked until the value falls below n."""
    i = np.asarray(i, dtype=np.uint64)
    h = 1
    while (1 << (2 * h)) < n:
        h += 1
    mask = np.uint64((1 << h) - 1)
    with np.errstate(over='ignore'):
        keys = [_splitmix64(np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15)
                            + np.uint64(epoch * 4 + j + 1)) for j in range(4)]
        x = i.copy()
        todo = np.ones(x.shape, dtype=bool)
        out = np.empty_like(x)
        while todo.any():
            L, R = x >> np.uint64(h), x & mask
            for k in keys:
                L, R = R, L ^ (_splitmix64(R ^ k) & mask)
            x = (L << np.uint64(h)) | R
            done = todo & (x < np.uint64(n))
            out[done] = x[done]
            todo &= ~done
    return out.astype(np.int64)


def batch_indices(t, n, B, seed):
    """Rows of minibatch number t (0-based) of the stream."""
    pos = np.arange(t * B, t * B + B, dtype=np.int64)
    epoch, i = pos // n, pos % n
    out = np.empty(B, dtype=np.int64)
    for e in np.unique(epoch):
        sel = epoch == e
        out[sel] = permute(i[sel], n, seed, int(e))
    return out


def optimiser_batches(iterations, log_every=10):
    """Stream batch number used by optimisation step k: the notebook evaluates
    training_loss() after steps 0, log_every, 2 log_every, ..., each drawing one
    batch from the same iterator."""
    k = np.arange(iterations)
    return k + (k + log_every - 1) // log_every if log_every else k


# ------------------------------------------------------------ kernel
def softplus(x):
    return np.logaddexp(0.0, x)


def inv_softplus(y):
    y = np.asarray(y, dtype=np.float64)
    return y + np.log(-np.expm1(-y))


def sigmoid(x):
    return 0.5 * (1.0 + np.tanh(0.5 * x))


def matern32(A, B, ls, var):
    """GPflow Matern32 K(A, B) and the pieces its derivatives need."""
    a, b = A / ls, B / ls
    r2 = np.sum(a * a, 1)[:, None] + np.sum(b * b, 1)[None, :] - 2.0 * a @ b.T
    r2 = np.maximum(r2, 0.0)
    r = np.sqrt(np.maximum(r2, 1e-36))
    e = np.exp(-SQRT3 * r)
    return var * (1.0 + SQRT3 * r) * e, e


# ------------------------------------------------------------ parameters
class Params:
    """Unconstrained SVGP state (what Adam updates)."""

    def __init__(self, Z, ls, var, noise, mean):
        M = len(Z)
        self.ls_raw = inv_softplus(np.asarray(ls, dtype=np.float64))
        self.var_raw = float(inv_softplus(var))
        self.lik_raw = float(inv_softplus(noise - LIK_LOWER))
        self.c = float(mean)
        self.Z = np.array(Z, dtype=np.float64)
        self.q_mu = np.zeros(M)
        self.S = np.eye(M)  # lower triangle used

    def flat(self):
        M = len(self.Z)
        tri = self.S[np.tril_indices(M)]
        return np.concatenate([self.ls_raw, [self.var_raw, self.lik_raw, self.c], self.Z.ravel(),
                               self.q_mu, tri])

    def set_flat(self, v):
        M = len(self.Z)
        self.ls_raw = v[:3].copy()
        self.var_raw, self.lik_raw, self.c = float(v[3]), float(v[4]), float(v[5])
        self.Z = v[6:6 + 3 * M].reshape(M, 3).copy()
        self.q_mu = v[6 + 3 * M:6 + 4 * M].copy()
        S = np.zeros((M, M))
        S[np.tril_indices(M)] = v[6 + 4 * M:]
        self.S = S

    def copy(self):
        p = Params.__new__(Params)
        p.ls_raw, p.var_raw, p.lik_raw, p.c = self.ls_raw.copy(), self.var_raw, self.lik_raw, self.c
        p.Z, p.q_mu, p.S = self.Z.copy(), self.q_mu.copy(), self.S.copy()
        return p


def constrained(p):
    return softplus(p.ls_raw), float(softplus(p.var_raw)), float(softplus(p.lik_raw)) + LIK_LOWER


# ------------------------------------------------------------ loss + gradient
def loss_and_grad(p, X, y, n, grad=True):
    """-ELBO of the minibatch (X [B x 3], y [B]) scaled to n data, and its
    gradient w.r.t. the unconstrained parameters in Params.flat() order."""
    ls, var, s2 = constrained(p)
    Z, q, S = p.Z, p.q_mu, np.tril(p.S)
    M, B = len(Z), len(y)
    Kuu, Eu = matern32(Z, Z, ls, var)
    L = np.linalg.cholesky(Kuu + JITTER * np.eye(M))
    Li = np.linalg.inv(L)
    Kuf, Ef = matern32(Z, X, ls, var)
    A = Li @ Kuf
    mu = p.c + A.T @ q
    SA = S.T @ A
    fv = var - np.sum(A * A, 0) + np.sum(SA * SA, 0)
    scale = n / B
    res = y - mu
    ve = -0.5 * np.log(2 * np.pi) - 0.5 * np.log(s2) - 0.5 * (res * res + fv) / s2
    d = np.diag(S)
    kl = 0.5 * (q @ q + np.sum(S * S) - M - np.sum(np.log(d * d)))
    loss = -(np.sum(ve) * scale - kl)
    if not grad:
        return loss
    g_mu = -scale * res / s2
    g_v = np.full(B, scale / (2 * s2))
    g_s2 = -scale * np.sum(-0.5 / s2 + 0.5 * (res * res + fv) / (s2 * s2))
    g_c = np.sum(g_mu)
    g_q = A @ g_mu + q
    Abar = np.outer(q, g_mu) - 2.0 * A * g_v + 2.0 * (S @ SA) * g_v
    Sbar = np.tril(2.0 * (A * g_v) @ SA.T + S - np.diag(1.0 / d))
    g_var = np.sum(g_v)
    Kfbar = Li.T @ Abar                      # dK_uf
    Lbar = np.tril(-Kfbar @ A.T)             # dL (A = L^-1 K_uf)
    P = np.tril(L.T @ Lbar)
    P[np.diag_indices(M)] *= 0.5
    Kbar = 0.5 * Li.T @ (P + P.T) @ Li       # dK_uu (symmetric)
    # kernel derivatives: dk/dr2 = -(3/2) var e;  r2 = sum_d (a_d - b_d)^2 / ls_d^2
    g_ls = np.zeros(3)
    g_Z = np.zeros((M, 3))
    for Kb, K, E, Bm, sym in ((Kfbar, Kuf, Ef, X, False), (Kbar, Kuu, Eu, Z, True)):
        W = Kb * (-1.5 * var) * E            # dL/dr2 per pair
        g_var += np.sum(Kb * K) / var
        for dd in range(3):
            diff = Z[:, dd][:, None] - Bm[:, dd][None, :]
            g_ls[dd] += np.sum(W * diff * diff) * (-2.0 / ls[dd] ** 3)
            gz = np.sum(W * diff, 1) * (2.0 / ls[dd] ** 2)
            g_Z[:, dd] += 2.0 * gz if sym else gz
    g = np.concatenate([g_ls * sigmoid(p.ls_raw), [g_var * sigmoid(p.var_raw),
                                                    g_s2 * sigmoid(p.lik_raw), g_c],
                        g_Z.ravel(), g_q, Sbar[np.tril_indices(M)]])
    return loss, g


def predict_f(p, xs):
    """GPflow SVGP.predict_f (whitened, full_cov=False): mean, variance."""
    ls, var, _ = constrained(p)
    M = len(p.Z)
    Kuu, _ = matern32(p.Z, p.Z, ls, var)
    L = np.linalg.cholesky(Kuu + JITTER * np.eye(M))
    Kus, _ = matern32(p.Z, xs, ls, var)
    A = np.linalg.solve(L, Kus)
    SA = np.tril(p.S).T @ A
    return p.c + A.T @ p.q_mu, var - np.sum(A * A, 0) + np.sum(SA * SA, 0)


# ------------------------------------------------------------ training
class Adam:
    def __init__(self, size, lr=1e-3, b1=0.9, b2=0.999, eps=1e-7):
        self.m, self.v, self.t = np.zeros(size), np.zeros(size), 0
        self.lr, self.b1, self.b2, self.eps = lr, b1, b2, eps

    def step(self, x, g):
        self.t += 1
        self.m = self.b1 * self.m + (1 - self.b1) * g
        self.v = self.b2 * self.v + (1 - self.b2) * g * g
        lr_t = self.lr * np.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        return x - lr_t * self.m / (np.sqrt(self.v) + self.eps)


def notebook_Z(x, M=50):
    """NB2: Z[:, d] = linspace(min x_d, max x_d, 50)."""
    return np.stack([np.linspace(np.min(x[:, d]), np.max(x[:, d]), M) for d in range(3)], 1)


def train(x, y, Z, ls, var, noise, mean, B=100, iterations=10000, seed=0, log_every=10):
    """NB2 SVGP(...): Adam on -ELBO over the deterministic minibatch stream.
    Returns (Params, elbo_log) -- elbo_log as the notebook records it
    (-training_loss on the next batch after every log_every-th step)."""
    n = len(y)
    p = Params(Z, ls, var, noise, mean)
    opt = Adam(len(p.flat()))
    used = optimiser_batches(iterations, log_every)
    log = []
    for k in range(iterations):
        idx = batch_indices(int(used[k]), n, B, seed)
        _, g = loss_and_grad(p, x[idx], y[idx], n)
        p.set_flat(opt.step(p.flat(), g))
        if log_every and k % log_every == 0:
            idx = batch_indices(int(used[k]) + 1, n, B, seed)
            log.append(-loss_and_grad(p, x[idx], y[idx], n, grad=False))
    return p, np.array(log)
