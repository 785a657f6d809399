"""Config-3-size T3 fixtures: the REFERENCE's own GPR3D(opt=True)
(GPR_CS2S3.py:143-191) on cells of n = 500 .. 3000 observations.

Run in the build container only (it reads /root/reference):
    python tests/golden/make_fit_large.py [--jobs 8]

For every cell the reference's GPR3D is run on a one-cell "day" whose
training set is the cell's observations (globals injected exactly as
make_golden.py does; the 300 km cKDTree query GPR:159 resolves the inputs),
once on the original observation order and on 4 random permutations of the
training set (the reference's chaotic stopping point moves with the
summation order).  Recorded per run: the 8-tuple, the number
of SMLII evaluations and the nlZ (oracle-free: the reference's own SMLII at
the run's hypers on the ORIGINAL order).  tests/test_gpu_fit_large.py judges
the GPU fit against runs 0-3 (the envelope) and uses run 4 as the held-out
sample of the reference's own noise.  Only numeric vectors are written
(fit_large.npz); no reference source enters the repo.
"""
import argparse
import os
import sys
from multiprocessing import Pool

os.environ['OPENBLAS_NUM_THREADS'] = '1'   # one single-threaded process per core

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

SIZES = (500, 500, 500, 1000, 1000, 1000, 1500, 1500, 2000, 2000, 3000)
NRUNS = 5          # run 0: original order; 1..4: permuted (4 = held out)
R_MAX = 275e3      # obs within 275 km: grid snapping never crosses the 300 km radius


def cell(k):
    import numpy as np
    from optimalinterpolation_amd import synthetic
    rng = np.random.default_rng(5000 + k)
    cx, cy = 4e6 + 1e5 * k, 3.5e6 - 7e4 * k
    x, z = synthetic.cell_obs(rng, cx, cy, SIZES[k], r_max=R_MAX)
    return np.array([[cx, cy]]), x, z


def run(job):
    k, r = job
    import numpy as np
    from make_golden import X0, cell_inputs, install_day, load_reference
    from optimalinterpolation_amd import synthetic
    ref = load_reference()
    X, x, z = cell(k)
    if r > 0:
        p = np.random.default_rng(900 + 31 * k + r).permutation(len(z))
        x, z = x[p], z[p]
    install_day(ref, X, x[:, 0].copy(), x[:, 1].copy(), x[:, 2].copy(), z.copy(), synthetic.PRIOR_MEAN)
    orig = ref['SMLII']
    count = [0]

    def counted(h, xx, yy, mX):
        count[0] += 1
        return orig(h, xx, yy, mX)
    ref['SMLII'] = counted
    t8 = np.array(ref['GPR3D'](0), dtype=float)          # opt=True, GPR:260
    ref['SMLII'] = orig
    inputs, outputs = cell_inputs(ref, 0)
    return k, r, t8, count[0], inputs, outputs


def main():
    import numpy as np
    import scipy
    from make_golden import REF, FIRST, LAST, load_reference, ragged
    ap = argparse.ArgumentParser()
    ap.add_argument('--jobs', type=int, default=8)
    ap.add_argument('--out', default=os.path.join(HERE, 'fit_large.npz'))
    ap.add_argument('--sizes', default='', help='comma list overriding SIZES (dry runs)')
    args = ap.parse_args()
    global SIZES
    if args.sizes:
        SIZES = tuple(int(v) for v in args.sizes.split(','))
    jobs = sorted([(k, r) for k in range(len(SIZES)) for r in range(NRUNS)], key=lambda j: -SIZES[j[0]])
    with Pool(args.jobs) as pool:
        res = {}
        for k, r, t8, ev, inp, out in pool.imap_unordered(run, jobs):
            res[(k, r)] = (t8, ev, inp, out)
            print(f"cell {k} (n={SIZES[k]}) run {r}: {ev} evals, fs {t8[0]:.10f}", flush=True)
    ref = load_reference()
    inx, iny, out8, evals, nlz = [], [], [], [], []
    for k in range(len(SIZES)):
        _, _, inp0, y0 = res[(k, 0)]
        assert len(y0) == SIZES[k]
        inx.append(inp0)
        iny.append(y0)
        mX = np.ones(len(y0)) * synthetic_mean()
        row8, rowe, rowf = [], [], []
        for r in range(NRUNS):
            t8, ev, _, _ = res[(k, r)]
            h = np.r_[np.log(t8[3:8]), np.log(.1)]
            f, _ = ref['SMLII'](h, inp0, y0, mX)    # the reference's nlZ on the original order
            row8.append(t8)
            rowe.append(ev)
            rowf.append(float(np.asarray(f).item()) if np.ndim(f) else float(f))
        out8.append(row8)
        evals.append(rowe)
        nlz.append(rowf)
    IX, offs = ragged(inx, 3)
    IY, _ = ragged(iny, 1)
    xs = np.array([[cell(k)[0][0, 0], cell(k)[0][0, 1], 4.0] for k in range(len(SIZES))])
    np.savez_compressed(args.out, x=IX, y=IY, offs=offs, xs=xs,
                        mean=synthetic_mean(), out8=np.array(out8), evals=np.array(evals),
                        nlz=np.array(nlz), sizes=np.array(SIZES), numpy=np.__version__,
                        scipy=scipy.__version__, ref=REF, lines=f'{FIRST}-{LAST}')


def synthetic_mean():
    from optimalinterpolation_amd import synthetic
    return synthetic.PRIOR_MEAN


if __name__ == '__main__':
    main()
