"""Golden fixtures for the Nystrom variant of the reference notebook
(GP_example.ipynb, abbreviated NB1), produced by running the REFERENCE's own
functions.  Run in the build container only (reads /root/reference):

    python tests/golden/make_nystrom_golden.py

The notebook cannot be executed as a whole (Basemap, netCDF4, data files and
a Mac data path), but its function definitions -- ``SGPkernel``, ``SMLII``,
``GPR``, ``Nystroem`` (code cell 1) -- are self-contained NumPy/SciPy.  This
script parses that cell, compiles only those four ``def`` blocks (AST), and
records inputs and outputs on synthetic cells with distinct, well separated
sites (the Nystrom formula divides by eigenvalues of a random-subset K_mm;
duplicated sites make those ~0 and the output rounding noise).  Only the
numeric vectors are committed (tests/golden/nystrom.npz).
"""
import ast
import json
import os
import sys

import numpy as np
import scipy
import scipy.optimize
from numpy.linalg import multi_dot as mdot
from scipy.spatial.distance import cdist, pdist, squareform

HERE = os.path.dirname(os.path.abspath(__file__))
NB = '/root/reference/GP_example.ipynb'
FUNCS = ('SGPkernel', 'SMLII', 'GPR', 'Nystroem')


def load_notebook_functions():
    cells = json.load(open(NB))['cells']
    src = ''.join(cells[1]['source'])
    # IPython magics (e.g. "%matplotlib inline") are not Python: blank them
    src = '\n'.join('' if ln.lstrip().startswith('%') else ln for ln in src.split('\n'))
    tree = ast.parse(src)
    keep = [node for node in tree.body if isinstance(node, ast.FunctionDef) and node.name in FUNCS]
    assert sorted(n.name for n in keep) == sorted(FUNCS)
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {'np': np, 'scipy': scipy, 'squareform': squareform, 'pdist': pdist, 'cdist': cdist,
          'mdot': mdot}
    exec(compile(mod, NB, 'exec'), ns)
    return ns


def cell_inputs(rng, n, spacing=25e3):
    """n distinct (x, y, t) sites around the origin on a 25 km grid x 9 days."""
    g = np.arange(-12, 13) * spacing
    sites = np.array([(a, b, t) for a in g for b in g for t in range(9)], dtype=np.float64)
    sel = rng.choice(len(sites), n, replace=False)
    x = sites[sel]
    y = (0.05 * np.sin(x[:, 0] / 2e5) * np.cos(x[:, 1] / 3e5) + 0.01 * (x[:, 2] - 4)
         + rng.normal(0.0, 0.02, n))
    return x, y


def main():
    ns = load_notebook_functions()
    rng = np.random.default_rng(2024)
    cases = [(120, 24), (200, 40), (300, 60), (64, 64), (257, 50)]
    hyps = [np.log([9e4, 7e4, 2.3, 8.7e-3, 4.3e-3]),
            np.log([6e4, 8e4, 4.0, 5e-3, 2e-3])]
    xs = np.array([[0.0, 0.0, 4.0]])
    X, Y, offs, Hs, Ms, nlz, grad, fs, sd, sprior = [], [], [0], [], [], [], [], [], [], []
    for n, M in cases:
        x, y = cell_inputs(rng, n)
        for h in hyps:
            f, g = ns['SMLII'](h, x, y, True, M)
            ell = list(np.exp(h[:3]))
            sf2, sn2 = np.exp(h[3]), np.exp(h[4])
            a, b, c = ns['GPR'](x, y, xs, ell=ell, sf2=sf2, sn2=sn2, mean=0.28, approx=True, M=M,
                                returnprior=True)
            X.append(x)
            Y.append(y)
            offs.append(offs[-1] + n)
            Hs.append(h)
            Ms.append(M)
            nlz.append(float(np.asarray(f).item()))
            grad.append(np.asarray(g, dtype=np.float64))
            fs.append(float(np.asarray(a).item()))
            sd.append(float(np.asarray(b).item()))
            sprior.append(float(c))
    np.savez_compressed(os.path.join(HERE, 'nystrom.npz'), x=np.concatenate(X), y=np.concatenate(Y),
                        offs=np.array(offs, dtype=np.int64), h=np.array(Hs), M=np.array(Ms),
                        xs=xs, mean=0.28, nlz=np.array(nlz), grad=np.array(grad), fs=np.array(fs),
                        sd=np.array(sd), sprior=np.array(sprior))
    print('wrote', len(nlz), 'cases')


if __name__ == '__main__':
    sys.exit(main())
