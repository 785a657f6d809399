# scipy CG driven by the GPU's n x n objective (OI_DEDUP=0) on one day-fixture
# cell, each evaluation also made by the CPU oracle (the reference's n x n
# algorithm): where do the two first disagree (value > 1e-8 rel, or finiteness)?
import os, sys, time, numpy as np
sys.path.insert(0, os.getcwd())
os.environ['OI_DEDUP'] = sys.argv[2] if len(sys.argv) > 2 else '0'
from scipy.optimize import minimize
from optimalinterpolation_amd import _lib
from oracle import gp_oracle as O
d = np.load('tests/golden/day_ref_fits.npz')
c = int(sys.argv[1]); a, b = d['offs'][c], d['offs'][c + 1]
x = d['x'].reshape(-1, 3)[a:b]; y = d['y'][a:b]; mean = float(d['mean']); mX = np.full(len(y), mean)
rows = []
def f(h):
    nlz, g, st = _lib.nlml_grad_batch(x, y, mX, np.array([0, len(y)]), h[None, :])
    fc, gc = O.neg_log_ml(h, x, y, mX)
    fc = float(np.asarray(fc).ravel()[0])
    rows.append((h.copy(), float(nlz[0]), fc, int(st[0])))
    return float(nlz[0]), np.asarray(g[0], float)
t = time.time()
r = minimize(f, np.array(O.X0_PRODUCTION), jac=True, method='CG')
print(f"cell {c} n={len(y)} OI_DEDUP={os.environ['OI_DEDUP']}: nfev {r.nfev} status {r.status} fun {r.fun} ({time.time()-t:.0f} s)")
first = None
for k, (h, fg, fc, st) in enumerate(rows):
    same = (np.isfinite(fg) == np.isfinite(fc)) and (not np.isfinite(fc) or abs(fg - fc) <= 1e-8 * abs(fc))
    if not same and first is None:
        first = k
    if not same and k < (first or 0) + 5:
        print(f"  eval {k}: h {np.round(h[:5], 4).tolist()} gpu {fg} oracle {fc} status {st}")
print('first disagreement', first, 'of', len(rows), '; inf evaluations gpu', sum(not np.isfinite(r_[1]) for r_ in rows),
      'oracle', sum(not np.isfinite(r_[2]) for r_ in rows))
