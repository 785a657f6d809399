"""GPU vs oracle divergence of the SVGP training over iterations (diagnostic)."""
import sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from oracle import svgp_oracle as O
from optimalinterpolation_amd import _lib, svgp

rng = np.random.default_rng(1)
def cell(n):
    x = np.stack([rng.uniform(-3e5, 3e5, n), rng.uniform(-3e5, 3e5, n), rng.integers(0, 9, n).astype(float)], 1)
    y = 0.3 + 0.05 * np.sin(x[:, 0] / 1e5) + 0.02 * np.cos(x[:, 1] / 7e4) + rng.normal(0, 0.02, n)
    return x, y
for n, M, B, iters in [(300, 12, 40, 1), (300, 12, 40, 15), (500, 20, 64, 200), (4600, 50, 100, 1000)]:
    x, y = cell(n)
    Z = O.notebook_Z(x, M)
    init = np.array([[25e3, 25e3, 1.0, 1.0, 0.1, 0.3]])
    xs = np.array([[1e4, -2e4, 4.0]])
    t = time.time()
    pred, st, params, elbo = _lib.svgp_batch(x, y, [0, n], Z[None], init, xs, batch=B, iterations=iters,
                                             log_every=10, seed=7, want_params=True)
    tg = time.time() - t
    t = time.time()
    p, log = O.train(x, y, Z, [25e3, 25e3, 1.0], 1.0, 0.1, 0.3, B=B, iterations=iters, seed=7)
    m, v = O.predict_f(p, xs)
    tc = time.time() - t
    th = p.flat()
    d = np.abs(params[0] - th) / np.maximum(1.0, np.abs(th))
    print(f"n={n} M={M} B={B} iters={iters}: status {st[0]} param max rel {d.max():.3e} (argmax {d.argmax()}), "
          f"elbo rel {np.max(np.abs(elbo[0] - log) / np.abs(log)):.3e}, pred {pred[0]} vs {m[0]:.10g} {v[0]:.10g}, "
          f"gpu {tg:.2f}s cpu {tc:.2f}s", flush=True)
