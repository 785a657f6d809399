"""Golden result for the notebook's Nystrom fit at its own scale (GP_example.ipynb
code cell 5: minimize(SMLII, x0, args=(inputs, outputs-mX, True, M=925),
method='CG', jac=True) then GPR(approx=True)), computed with the oracle --
oracle/nystrom_oracle.py is bit-for-bit equal to the notebook's functions
(tests/test_oracle_golden.py) -- and scipy 1.15's CG, on one synthetic cell of
n = 4600 distinct 25 km x 9-day sites (well conditioned).  ~2 min of CPU:

    python tests/golden/make_nystrom_fit_golden.py
"""
import os
import sys

import numpy as np
import scipy.optimize

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import nystrom_oracle as N  # noqa: E402


def cell():
    rng = np.random.default_rng(5)
    g = np.arange(-12, 13) * 25e3
    sites = np.array([(a, b, t) for a in g for b in g for t in range(9)], dtype=np.float64)
    n = 4600
    x = sites[rng.choice(len(sites), n, replace=False)]
    y = 0.05 * np.sin(x[:, 0] / 2e5) + 0.01 * (x[:, 2] - 4) + rng.normal(0, 0.02, n)
    return x, y


def main():
    x, y = cell()
    M, mean = 925, 0.28
    x0 = [np.log(25e3), np.log(25e3), np.log(1.), np.log(1.), np.log(.1)]

    def f(h):
        a, b = N.neg_log_ml(h, x, y, M)
        return float(np.asarray(a).item()), b

    r = scipy.optimize.minimize(f, x0=x0, method='CG', jac=True)
    ell = list(np.exp(r.x[:3]))
    fs, sd, sp = N.predict(x, y, np.array([[0.0, 0.0, 4.0]]), ell, np.exp(r.x[3]), np.exp(r.x[4]),
                           mean, M)
    np.savez_compressed(os.path.join(HERE, 'nystrom_fit.npz'), x=x, y=y, M=M, mean=mean,
                        x0=np.array(x0), hyp=r.x, fun=r.fun, nit=r.nit, nfev=r.nfev, status=r.status,
                        fs=float(np.asarray(fs).item()), sd=float(np.asarray(sd).item()), sprior=float(sp))
    print('nit', r.nit, 'nfev', r.nfev, 'status', r.status, 'x', np.exp(r.x), 'fs', fs, 'sd', sd)


if __name__ == '__main__':
    main()
