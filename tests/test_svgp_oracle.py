"""The SVGP oracle (oracle/svgp_oracle.py, GPflow SVGP of dev/sparseGP_example.ipynb
restated) checked on its own: hand-derived gradient vs central finite
differences and vs torch autograd of an independent torch restatement of the
same ELBO; the minibatch permutation is a bijection; Adam matches its formula."""
import numpy as np
import pytest

from oracle import svgp_oracle as O


def _cell(rng, n=300):
    x = np.stack([rng.uniform(-3e5, 3e5, n), rng.uniform(-3e5, 3e5, n),
                  rng.integers(0, 9, n).astype(float)], 1)
    y = 0.3 + 0.05 * np.sin(x[:, 0] / 1e5) + rng.normal(0, 0.02, n)
    return x, y


def _state(rng, M=12):
    x, y = _cell(rng)
    p = O.Params(O.notebook_Z(x, M), [9e4, 7e4, 2.0], 0.01, 0.004, 0.3)
    # move away from the initial point so every gradient term is exercised
    p.q_mu = rng.normal(0, 0.1, M)
    p.S = np.tril(rng.normal(0, 0.1, (M, M))) + np.eye(M)
    p.Z = p.Z + rng.normal(0, 2e4, p.Z.shape) * np.array([1, 1, 0.0001])
    return x, y, p


def test_permutation_is_bijection():
    for n in (1, 7, 100, 4600, 4097):
        for e in (0, 3):
            v = O.permute(np.arange(n), n, seed=11, epoch=e)
            assert np.array_equal(np.sort(v), np.arange(n))
    a = O.permute(np.arange(500), 500, 1, 0)
    assert not np.array_equal(a, O.permute(np.arange(500), 500, 2, 0))
    assert not np.array_equal(a, O.permute(np.arange(500), 500, 1, 1))


def test_optimiser_batch_schedule():
    # step 0 uses batch 0, the log after it batch 1, steps 1..9 batches 2..10,
    # step 10 batch 11, its log 12, step 11 batch 13
    u = O.optimiser_batches(12, 10)
    assert list(u) == [0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13]


def test_gradient_finite_differences():
    rng = np.random.default_rng(3)
    x, y, p = _state(rng)
    idx = O.batch_indices(0, len(y), 40, seed=5)
    f0, g = O.loss_and_grad(p, x[idx], y[idx], len(y))
    v0 = p.flat()
    k = np.arange(len(v0))
    for j in k[::3]:
        h = 1e-6 * max(1.0, abs(v0[j]))
        q = p.copy()
        v = v0.copy(); v[j] += h; q.set_flat(v)
        fp = O.loss_and_grad(q, x[idx], y[idx], len(y), grad=False)
        v = v0.copy(); v[j] -= h; q.set_flat(v)
        fm = O.loss_and_grad(q, x[idx], y[idx], len(y), grad=False)
        fd = (fp - fm) / (2 * h)
        assert abs(fd - g[j]) <= 1e-5 * max(1.0, abs(g[j]), abs(f0) * 1e-6), (j, fd, g[j])


def test_gradient_vs_torch_autograd():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(4)
    x, y, p = _state(rng)
    idx = O.batch_indices(2, len(y), 50, seed=1)
    X, Y, n = x[idx], y[idx], len(y)
    _, g = O.loss_and_grad(p, X, Y, n)
    M = len(p.Z)
    t = lambda a: torch.tensor(a, dtype=torch.float64, requires_grad=True)
    ls_raw, var_raw, lik_raw, c = t(p.ls_raw), t(p.var_raw), t(p.lik_raw), t(p.c)
    Z, q = t(p.Z), t(p.q_mu)
    tri = t(p.S[np.tril_indices(M)])
    Xt, Yt = torch.tensor(X), torch.tensor(Y)
    ls = torch.nn.functional.softplus(ls_raw)
    var = torch.nn.functional.softplus(var_raw)
    s2 = torch.nn.functional.softplus(lik_raw) + 1e-6
    S = torch.zeros(M, M, dtype=torch.float64)
    S = S.index_put((torch.tensor(np.tril_indices(M)[0]), torch.tensor(np.tril_indices(M)[1])), tri)

    def K(A, B):
        a, b = A / ls, B / ls
        r2 = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
        r = torch.sqrt(torch.clamp(torch.clamp(r2, min=0.0), min=1e-36))
        return var * (1 + np.sqrt(3) * r) * torch.exp(-np.sqrt(3) * r)

    L = torch.linalg.cholesky(K(Z, Z) + 1e-6 * torch.eye(M, dtype=torch.float64))
    A = torch.linalg.solve_triangular(L, K(Z, Xt), upper=False)
    mu = c + A.T @ q
    SA = S.T @ A
    fv = var - (A * A).sum(0) + (SA * SA).sum(0)
    ve = -0.5 * np.log(2 * np.pi) - 0.5 * torch.log(s2) - 0.5 * ((Yt - mu) ** 2 + fv) / s2
    kl = 0.5 * (q @ q + (S * S).sum() - M - torch.log(torch.diagonal(S) ** 2).sum())
    loss = -(ve.sum() * n / len(Y) - kl)
    loss.backward()
    tg = np.concatenate([ls_raw.grad.numpy(), [var_raw.grad.item(), lik_raw.grad.item(), c.grad.item()],
                         Z.grad.numpy().ravel(), q.grad.numpy(), tri.grad.numpy()])
    assert np.allclose(g, tg, rtol=1e-7, atol=1e-7 * np.abs(tg).max()), np.abs(g - tg).max()


def test_adam_formula():
    a = O.Adam(2)
    x = np.array([1.0, -2.0])
    g = np.array([0.5, -0.25])
    x1 = a.step(x, g)
    # first step: m = .1 g, v = .001 g^2, lr_t = 1e-3 sqrt(.001)/.1
    lr_t = 1e-3 * np.sqrt(1 - 0.999) / (1 - 0.9)
    assert np.allclose(x1, x - lr_t * (0.1 * g) / (np.sqrt(0.001 * g * g) + 1e-7))


def test_training_improves_elbo():
    rng = np.random.default_rng(8)
    x, y = _cell(rng, 400)
    p, log = O.train(x, y, O.notebook_Z(x, 10), [25e3, 25e3, 1.0], 1.0, 0.1, 0.3, B=50,
                     iterations=300, seed=3)
    assert np.all(np.isfinite(log)) and log[-5:].mean() > log[:5].mean()
    m, v = O.predict_f(p, np.array([[0.0, 0.0, 4.0]]))
    assert np.isfinite(m).all() and (v > 0).all()
