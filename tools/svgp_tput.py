"""SVGP kernel: time per step vs threads per cell and number of cells (diagnostic)."""
import os, sys, time
sys.path.insert(0, '/root/repo')
import numpy as np
from oracle import svgp_oracle as O
from optimalinterpolation_amd import _lib

rng = np.random.default_rng(1)
n, M, B = 4600, 50, 100
def cells(k):
    xs, ys = [], []
    for _ in range(k):
        x = np.stack([rng.uniform(-3e5, 3e5, n), rng.uniform(-3e5, 3e5, n), rng.integers(0, 9, n).astype(float)], 1)
        xs.append(x); ys.append(0.3 + 0.05 * np.sin(x[:, 0] / 1e5) + rng.normal(0, 0.02, n))
    return np.concatenate(xs), np.concatenate(ys), np.arange(k + 1) * n, np.stack([O.notebook_Z(x, M) for x in xs])
X, Y, offs, Z = cells(int(sys.argv[2]) if len(sys.argv) > 2 else 256)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for k in (1, 256, len(offs) - 1):
    if k > len(offs) - 1: continue
    init = np.tile([25e3, 25e3, 1.0, 1.0, 0.1, 0.3], (k, 1))
    xs = np.tile([[1e4, -2e4, 4.0]], (k, 1))
    _lib.svgp_batch(X[:k * n], Y[:k * n], offs[:k + 1], Z[:k], init, xs, batch=B, iterations=2)  # warm
    t = time.time()
    pred, st, _, _ = _lib.svgp_batch(X[:k * n], Y[:k * n], offs[:k + 1], Z[:k], init, xs, batch=B, iterations=iters)
    dt = time.time() - t
    print(f"threads {os.environ.get('OI_SVGP_THREADS', '256')} cells {k} iters {iters}: {dt:.3f} s, "
          f"{dt / iters * 1e6:.1f} us/step, {k * iters / dt:.0f} cell-steps/s, status {st.sum()}", flush=True)
