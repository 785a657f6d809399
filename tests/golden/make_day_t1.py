"""T1 noise fixture on the HEADLINE's own cells (VERDICT r5 "next" item 1):
the REFERENCE's own SMLII (GPR_CS2S3.py:107-141) on the 360 cells of
day_ref_fits.npz, in each of the 5 observation orders those fits used, at two
hyper points per cell:

  point 0: x0 of the production script (GPR:217), where every CG run starts;
  point 1: the hypers the reference's run 0 ended at (out8[:, 0, 3:8]).

The spread of the reference's objective over observation orders at FIXED
hypers is the rounding noise the chaotic CG feeds on; the
GPU's own distance to run 0 at the same points is measured against it by
tests/test_gpu_day_t1.py.

Orders are regenerated exactly as make_day_fits.py made them (the day cell's
observations, run r > 0 permuted by default_rng(7000 + 13 idx + r), then the
reference's cKDTree query at 325 km, GPR:159-161); order 0 is asserted equal
to the fixture's stored inputs.  Writes day_ref_t1.npz (numeric arrays
only).  Build container only (reads /root/reference):
    python tests/golden/make_day_t1.py [--jobs 7] [--extend]
"""
import argparse
import os
import sys
from multiprocessing import Pool

os.environ['OPENBLAS_NUM_THREADS'] = '1'

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

NRUNS = 5
_STATE = {}


def state():
    if not _STATE:
        import numpy as np
        from make_day_fits import day
        _STATE['fx'] = dict(np.load(os.path.join(HERE, 'day_ref_fits.npz')))
        _STATE['day'] = day()
    return _STATE['fx'], _STATE['day']


def order_inputs(ref, d, idx, r, radius_km):
    """The inputs GPR3D saw in run r of make_day_fits.run (same permutation, same query)."""
    import numpy as np
    from make_golden import cell_inputs, install_day
    x, z, xs = d.cell(idx)
    n = len(z)
    if r > 0:
        p = np.random.default_rng(7000 + 13 * idx + r).permutation(n)
        x, z = x[p], z[p]
    install_day(ref, xs[:, :2].copy(), x[:, 0].copy(), x[:, 1].copy(), x[:, 2].copy(), z.copy(), d.mean)
    ref['radius'] = radius_km
    return cell_inputs(ref, 0)


def job(args):
    k, r = args
    import numpy as np
    from make_golden import X0, load_reference
    fx, d = state()
    ref = load_reference()
    idx = int(fx['cells'][k])
    inp, out = order_inputs(ref, d, idx, r, int(fx['radius_km']))
    if r == 0:
        a, b = fx['offs'][k], fx['offs'][k + 1]
        assert np.array_equal(inp, fx['x'].reshape(-1, 3)[a:b]) and np.array_equal(out, fx['y'][a:b]), k
    pts = [np.array(X0), np.r_[np.log(fx['out8'][k, 0, 3:8]), np.log(.1)]]
    res = np.full((2, 7), np.nan)
    mX = np.ones(len(out)) * float(fx['mean'])
    for p, h in enumerate(pts):
        if not np.all(np.isfinite(h)):
            continue
        f, g = ref['SMLII'](h, inp, out, mX)
        res[p, 0] = float(np.asarray(f).item()) if np.ndim(f) else float(f)
        res[p, 1:] = np.asarray(g, float)
    return k, r, res, np.array(pts)


def main():
    import numpy as np
    import scipy
    from make_golden import FIRST, LAST, REF
    ap = argparse.ArgumentParser()
    ap.add_argument('--jobs', type=int, default=7)
    ap.add_argument('--out', default=os.path.join(HERE, 'day_ref_t1.npz'))
    ap.add_argument('--extend', action='store_true',
                    help='keep the cells already in --out and compute only the cells day_ref_fits.npz added since')
    args = ap.parse_args()
    fx, _ = state()
    sizes = fx['sizes']
    k0 = 0
    if args.extend:
        old = dict(np.load(args.out))
        k0 = len(old['cells'])
        assert np.array_equal(old['cells'], fx['cells'][:k0]), "day_ref_t1.npz is not a prefix of day_ref_fits.npz"
    jobs = sorted([(k, r) for k in range(k0, len(sizes)) for r in range(NRUNS)], key=lambda j: -int(sizes[j[0]]))
    nlz = np.full((len(sizes), 2, NRUNS), np.nan)
    grad = np.full((len(sizes), 2, NRUNS, 6), np.nan)
    hyp = np.full((len(sizes), 2, 6), np.nan)
    if args.extend:
        nlz[:k0], grad[:k0], hyp[:k0] = old['nlz'], old['grad'], old['hyp']
    with Pool(args.jobs) as pool:
        for i, (k, r, res, pts) in enumerate(pool.imap_unordered(job, jobs)):
            nlz[k, :, r] = res[:, 0]
            grad[k, :, r] = res[:, 1:]
            hyp[k] = pts
            if i % 100 == 0:
                print(f"{i}/{len(jobs)} (cell {k}, n={int(sizes[k])}, order {r})", flush=True)
    np.savez_compressed(args.out, cells=fx['cells'], sizes=sizes, hyp=hyp, nlz=nlz, grad=grad,
                        numpy=np.__version__, scipy=scipy.__version__, ref=REF, lines=f'{FIRST}-{LAST}')
    print(f"wrote {args.out}: {len(sizes)} cells x 2 points x {NRUNS} orders", flush=True)


if __name__ == '__main__':
    main()
