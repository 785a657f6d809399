"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the build container only (it reads /root/reference, which is absent on
the GPU box):  ``python tests/golden/make_golden.py``

The reference module as a whole cannot be imported under Python 3
(SyntaxError at GPR_CS2S3.py:317, Python-2 izip_longest at :270,:325,
module-level reads of absent data files at :203-214, mpi4py/astropy missing),
but its hot-path functions -- ``SGPkernel``, ``SMLII``, ``GPR3D``
(GPR_CS2S3.py:78-191) -- execute fine.  This script compiles exactly that
line range from the reference file at run time, injects the module globals
``GPR3D`` reads (GPR_CS2S3.py:159-172) for small synthetic "days", and
records inputs and outputs.  No reference source is copied into the repo:
only the numeric vectors below are committed.

Fixtures written (np.savez_compressed, no pickles):
  smlii.npz    nlZ / dnlZ of SMLII at fixed hyper-parameters (T1 pin)
  cg.npz       every SMLII call scipy's CG made inside GPR3D's minimize
               (x, f, g) + final x / nit / nfev / status           (T2 pin)
  gpr3d.npz    GPR3D(index, opt=True) 8-tuples and GPR3D(index, opt=False)
               2-tuples on a synthetic mini-day, with the resolved neighbour
               inputs in query_ball_point order                    (T1/T3 pin)
  predict64.npz 64 cells x n=200, GPR3D(opt=False) with fixed hypers
"""
import os
import sys

import numpy as np
import scipy
import scipy.optimize
import scipy.spatial
from scipy.spatial.distance import cdist, pdist, squareform

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from optimalinterpolation_amd import synthetic  # noqa: E402

REF = '/root/reference/2021_paper_production/GPR_CS2S3.py'
FIRST, LAST = 78, 191          # SGPkernel .. end of GPR3D


def load_reference():
    lines = open(REF).readlines()
    assert lines[FIRST - 1].startswith('def SGPkernel'), lines[FIRST - 1]
    assert lines[LAST - 1].strip() == 'return np.nan,np.nan', lines[LAST - 1]
    ns = {'np': np, 'scipy': scipy, 'squareform': squareform, 'pdist': pdist,
          'cdist': cdist}
    code = compile(''.join(lines[FIRST - 1:LAST]), REF, 'exec')
    exec(code, ns)
    return ns


X0 = [np.log(25 * 1000), np.log(25 * 1000), np.log(1.), np.log(1.), np.log(1.), np.log(.1)]  # GPR:217


def ragged(list_of_arrays, width):
    offs = [0]
    for a in list_of_arrays:
        offs.append(offs[-1] + len(a))
    cat = (np.concatenate([np.asarray(a, float).reshape(-1, width) for a in list_of_arrays])
           if list_of_arrays else np.zeros((0, width)))
    if width == 1:
        cat = cat.reshape(-1)
    return cat, np.array(offs, dtype=np.int64)


def with_duplicates(rng, x, y, frac=0.1):
    """Append exact duplicate sites (same x, y, t) with fresh noise."""
    k = max(1, int(frac * len(y)))
    idx = rng.integers(0, len(y), k)
    return (np.concatenate([x, x[idx]]),
            np.concatenate([y, y[idx] + rng.normal(0, 0.02, k)]))


def gen_smlii(ref, rng):
    sets = []
    for n in [0, 1, 2, 3, 50, 200, 500]:
        x, y = synthetic.cell_obs(rng, 4e6, 4e6, n)
        if n == 500:
            x, y = with_duplicates(rng, x, y)
        sets.append((x, y))
    hyps = [
        np.array(X0),
        np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), np.log(.1)]),
        np.array([np.log(1.2e5), np.log(2.1e5), np.log(4.), np.log(2e-2), np.log(3e-3), 0.3]),
        np.array([np.log(6e4), np.log(4e4), np.log(1.5), np.log(1e-3), np.log(1e-4), -1.0]),
    ]
    xs, ys, H, F, G, ks = [], [], [], [], [], []
    mean = synthetic.PRIOR_MEAN
    for (x, y) in sets:
        for h in hyps:
            mX = np.ones(len(y)) * mean
            f, g = ref['SMLII'](h, x, y, mX)
            xs.append(x)
            ys.append(y)
            H.append(h)
            F.append(float(np.asarray(f).item()) if np.ndim(f) else float(f))
            G.append(np.asarray(g, float))
    X, offs = ragged(xs, 3)
    Y, _ = ragged(ys, 1)
    return dict(x=X, y=Y, offs=offs, mean=mean, h=np.array(H), nlZ=np.array(F), g=np.array(G))


def mini_day(rng, sizes, spacing=700e3, origin=(0.6e6, 0.6e6), per_row=8):
    """Cells with disjoint 300 km discs; obs only inside r <= 275 km so that
    grid snapping never moves one across the 300 km query radius."""
    cen, xtr, ytr, ttr, zz = [], [], [], [], []
    for c, n in enumerate(sizes):
        cx = origin[0] + (c % per_row) * spacing
        cy = origin[1] + (c // per_row) * spacing
        cen.append((cx, cy))
        x, z = synthetic.cell_obs(rng, cx, cy, int(n), r_max=275e3)
        xtr.append(x[:, 0])
        ytr.append(x[:, 1])
        ttr.append(x[:, 2])
        zz.append(z)
    return (np.array(cen), np.concatenate(xtr), np.concatenate(ytr),
            np.concatenate(ttr), np.concatenate(zz))


def install_day(ref, X, x_train, y_train, t_train, z, mean):
    ref.update(X=X, x_train=x_train, y_train=y_train, t_train=t_train, z=z,
               radius=300, mean=mean, T_mid=4, x0=X0,
               X_tree=scipy.spatial.cKDTree(np.array([x_train, y_train]).T))


def cell_inputs(ref, index):
    ID = ref['X_tree'].query_ball_point(x=ref['X'][index, :], r=ref['radius'] * 1000)
    inputs = np.array([ref['x_train'][ID], ref['y_train'][ID], ref['t_train'][ID]]).T.reshape(-1, 3)
    return inputs, ref['z'][ID]


def gen_cg_and_gpr3d(ref, rng):
    sizes = [0, 1, 2, 3, 5, 12, 20, 50, 100, 150, 200, 300]
    mean = synthetic.PRIOR_MEAN
    X, x_train, y_train, t_train, z = mini_day(rng, sizes)
    install_day(ref, X, x_train, y_train, t_train, z, mean)
    orig = ref['SMLII']
    tr_x, tr_f, tr_g, tr_offs = [], [], [], [0]
    res_x, res_nit, res_nfev, res_status, out8, inx, iny = [], [], [], [], [], [], []
    for index in range(len(sizes)):
        inputs, outputs = cell_inputs(ref, index)
        assert len(outputs) == sizes[index], (index, len(outputs), sizes[index])
        calls = []

        def rec(h, x, y, mX):
            f, g = orig(h, x, y, mX)
            calls.append((np.array(h, float).copy(),
                          float(np.asarray(f).item()) if np.ndim(f) else float(f),
                          np.array(g, float).copy()))
            return f, g
        ref['SMLII'] = rec
        t8 = ref['GPR3D'](index)                 # opt=True, GPR:260
        ref['SMLII'] = orig
        # the same minimize call GPR3D makes (GPR:166), to capture nit/status
        mX = np.ones(len(outputs)) * mean
        res = scipy.optimize.minimize(orig, x0=X0, args=(inputs, outputs, mX), method='CG', jac=True)
        assert np.array_equal(np.exp(res.x)[:5], np.array(t8[3:8], float)), index
        for (h, f, g) in calls:
            tr_x.append(h)
            tr_f.append(f)
            tr_g.append(g)
        tr_offs.append(tr_offs[-1] + len(calls))
        res_x.append(res.x)
        res_nit.append(res.nit)
        res_nfev.append(res.nfev)
        res_status.append(res.status)
        out8.append(np.array(t8, dtype=float))
        inx.append(inputs)
        iny.append(outputs)
    IX, ioffs = ragged(inx, 3)
    IY, _ = ragged(iny, 1)
    cg = dict(x=IX, y=IY, offs=ioffs, mean=mean, x0=np.array(X0),
              trace_x=np.array(tr_x), trace_f=np.array(tr_f), trace_g=np.array(tr_g),
              trace_offs=np.array(tr_offs, dtype=np.int64),
              res_x=np.array(res_x), res_nit=np.array(res_nit), res_nfev=np.array(res_nfev),
              res_status=np.array(res_status))
    # pass 2 on the same day: smoothed hypers are given (GPR:313-315)
    out8a = np.array(out8)
    hyp = np.nan_to_num(out8a[:, 3:8], nan=1.0)
    hyp = hyp * np.exp(rng.normal(0, 0.1, hyp.shape))
    ref.update(ellXs=hyp[:, 0:3].copy(), sf2xs=hyp[:, 3].copy(), sn2xs=hyp[:, 4].copy())
    out2 = np.array([np.array(ref['GPR3D'](i, opt=False), dtype=float) for i in range(len(sizes))])
    g3 = dict(x=IX, y=IY, offs=ioffs, mean=mean, xs=np.column_stack([X, np.full(len(X), 4.0)]),
              out8=out8a, hyp2=hyp, out2=out2)
    return cg, g3


def gen_predict64(ref, rng):
    sizes = [200] * 64
    mean = synthetic.PRIOR_MEAN
    X, x_train, y_train, t_train, z = mini_day(rng, sizes)
    install_day(ref, X, x_train, y_train, t_train, z, mean)
    hyp = np.tile(np.array(synthetic.FIXED_HYPERS), (64, 1)) * np.exp(rng.normal(0, 0.05, (64, 5)))
    ref.update(ellXs=hyp[:, 0:3].copy(), sf2xs=hyp[:, 3].copy(), sn2xs=hyp[:, 4].copy())
    inx, iny, out2 = [], [], []
    for i in range(64):
        a, b = cell_inputs(ref, i)
        inx.append(a)
        iny.append(b)
        out2.append(np.array(ref['GPR3D'](i, opt=False), dtype=float))
    IX, ioffs = ragged(inx, 3)
    IY, _ = ragged(iny, 1)
    return dict(x=IX, y=IY, offs=ioffs, mean=mean, xs=np.column_stack([X, np.full(64, 4.0)]),
                hyp=hyp, out2=np.array(out2))


def main():
    ref = load_reference()
    meta = dict(numpy=np.__version__, scipy=scipy.__version__, ref=REF, lines=f'{FIRST}-{LAST}')
    np.savez_compressed(os.path.join(HERE, 'smlii.npz'), **gen_smlii(ref, np.random.default_rng(11)), **meta)
    cg, g3 = gen_cg_and_gpr3d(ref, np.random.default_rng(12))
    np.savez_compressed(os.path.join(HERE, 'cg.npz'), **cg, **meta)
    np.savez_compressed(os.path.join(HERE, 'gpr3d.npz'), **g3, **meta)
    np.savez_compressed(os.path.join(HERE, 'predict64.npz'), **gen_predict64(ref, np.random.default_rng(13)), **meta)
    print('wrote fixtures to', HERE)


if __name__ == '__main__':
    main()
