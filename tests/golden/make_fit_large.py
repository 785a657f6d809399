"""Config-3/5-size T3 fixtures: the REFERENCE's own GPR3D(opt=True)
(GPR_CS2S3.py:143-191) on cells of n = 500 .. 5000 observations (config 3
draws n from 300..3000, config 5 up to 5000): 27 cells, three in every
500-wide bucket from 500 to 5000.

Run in the build container only (it reads /root/reference):
    python tests/golden/make_fit_large.py [--jobs 8] [--merge]

--merge keeps the cells of an existing fit_large.npz whose size matches
(round 2 produced the first 11) and runs only the new ones; every finished
(cell, run) is also cached under tests/golden/_fit_cache/ (git-ignored), so
an interrupted generation resumes where it stopped.  An n = 5000 fit is
~150 SMLII calls of ~17 s each on one core.

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

SIZES = (500, 500, 500, 1000, 1000, 1000, 1500, 1500, 2000, 2000, 3000,      # round 2
         1700, 2300, 2600, 2800, 2950, 3250, 3450, 3600, 3800, 3950,         # round 3
         4000, 4250, 4450, 4600, 4800, 5000)
CACHE = os.path.join(HERE, '_fit_cache')
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
    import time
    import numpy as np
    path = os.path.join(CACHE, f'k{k}_n{SIZES[k]}_r{r}.npz')
    if os.path.exists(path):
        d = np.load(path)
        return k, r, d['t8'], int(d['ev']), d['inp'], d['out'], float(d['sec'])
    t0 = time.time()
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
    sec = time.time() - t0
    os.makedirs(CACHE, exist_ok=True)
    np.savez(path + '.tmp.npz', t8=t8, ev=count[0], inp=inputs, out=outputs, sec=sec)
    os.replace(path + '.tmp.npz', path)
    return k, r, t8, count[0], inputs, outputs, sec


def nlz_job(job):
    """The reference's own SMLII (GPR:107-141) at run r's hypers, on the
    ORIGINAL observation order of cell k."""
    k, t8, inp0, y0 = job
    import numpy as np
    from make_golden import load_reference
    ref = load_reference()
    mX = np.ones(len(y0)) * synthetic_mean()
    h = np.r_[np.log(t8[3:8]), np.log(.1)]
    f, _ = ref['SMLII'](h, inp0, y0, mX)
    return float(np.asarray(f).item()) if np.ndim(f) else float(f)


def main():
    import numpy as np
    import scipy
    from make_golden import REF, FIRST, LAST, ragged
    ap = argparse.ArgumentParser()
    ap.add_argument('--jobs', type=int, default=8)
    ap.add_argument('--out', default=os.path.join(HERE, 'fit_large.npz'))
    ap.add_argument('--sizes', default='', help='comma list overriding SIZES (dry runs)')
    ap.add_argument('--reverse', action='store_true',
                    help='smallest cells first (a second generator sharing the cache works from the other end)')
    ap.add_argument('--merge', nargs='?', const='', default=None,
                    help='reuse the cells of an existing fixture (default: --out) whose sizes match')
    ap.add_argument('--partial', action='store_true',
                    help='write the fixture from the cells whose runs are all finished (merged or cached); '
                         'run nothing new')
    args = ap.parse_args()
    global SIZES
    if args.sizes:
        SIZES = tuple(int(v) for v in args.sizes.split(','))
    res = {}
    merge_from = (args.merge or args.out) if args.merge is not None else None
    if merge_from and os.path.exists(merge_from):
        old = np.load(merge_from)
        osz, ooffs = old['sizes'], old['offs']
        ox, oy = old['x'].reshape(-1, 3), old['y']
        for k in range(min(len(osz), len(SIZES))):
            if osz[k] != SIZES[k]:
                break
            a, b = ooffs[k], ooffs[k + 1]
            for r in range(NRUNS):
                sec = float(old['sec'][k, r]) if 'sec' in old.files else float('nan')
                res[(k, r)] = (old['out8'][k, r], int(old['evals'][k, r]), ox[a:b], oy[a:b], sec)
        print(f"merged {len(res) // NRUNS} cells from {merge_from}", flush=True)
    jobs = sorted([(k, r) for k in range(len(SIZES)) for r in range(NRUNS) if (k, r) not in res],
                  key=lambda j: SIZES[j[0]] if args.reverse else -SIZES[j[0]])
    if args.partial:
        jobs = [(k, r) for k, r in jobs if os.path.exists(os.path.join(CACHE, f'k{k}_n{SIZES[k]}_r{r}.npz'))]
    with Pool(args.jobs) as pool:
        for k, r, t8, ev, inp, out, sec in pool.imap_unordered(run, jobs):
            res[(k, r)] = (t8, ev, inp, out, sec)
            print(f"cell {k} (n={SIZES[k]}) run {r}: {ev} evals, fs {t8[0]:.10f}, {sec:.0f} s", flush=True)
    cells = [k for k in range(len(SIZES)) if all((k, r) in res for r in range(NRUNS))]
    if len(cells) < len(SIZES):
        print(f"partial fixture: {len(cells)} of {len(SIZES)} cells complete", flush=True)
    nlz_jobs = [(k, res[(k, r)][0], res[(k, 0)][2], res[(k, 0)][3]) for k in cells for r in range(NRUNS)]
    with Pool(args.jobs) as pool:
        nlz_all = pool.map(nlz_job, nlz_jobs)
    inx, iny, out8, evals, nlz, secs = [], [], [], [], [], []
    for ci, k in enumerate(cells):
        _, _, inp0, y0, _ = res[(k, 0)]
        assert len(y0) == SIZES[k]
        inx.append(inp0)
        iny.append(y0)
        row8, rowe, rowf, rows = [], [], [], []
        for r in range(NRUNS):
            t8, ev, _, _, sec = res[(k, r)]
            rows.append(sec)
            row8.append(t8)
            rowe.append(ev)
            rowf.append(nlz_all[ci * NRUNS + r])    # the reference's nlZ on the original order
        out8.append(row8)
        evals.append(rowe)
        nlz.append(rowf)
        secs.append(rows)
    IX, offs = ragged(inx, 3)
    IY, _ = ragged(iny, 1)
    xs = np.array([[cell(k)[0][0, 0], cell(k)[0][0, 1], 4.0] for k in cells])
    np.savez_compressed(args.out, x=IX, y=IY, offs=offs, xs=xs,
                        mean=synthetic_mean(), out8=np.array(out8), evals=np.array(evals),
                        nlz=np.array(nlz), sizes=np.array([SIZES[k] for k in cells]), sec=np.array(secs),
                        numpy=np.__version__,
                        scipy=scipy.__version__, ref=REF, lines=f'{FIRST}-{LAST}')


def synthetic_mean():
    from optimalinterpolation_amd import synthetic
    return synthetic.PRIOR_MEAN


if __name__ == '__main__':
    main()
