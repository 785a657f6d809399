"""Benchmark: grid-cells/s for the full per-cell GP fit + predict (GPR3D,
opt=True) on the synthetic 25 km pan-Arctic day, fp64 (BASELINE.json).

Default workload `day` (config 3 at N = 1, config 4 at N > 1): the synthetic
day -- 9997 cells, n ~ U{300..3000} observations each -- is
split over the N ranks by LPT on the cost model E(n) n^3 (driver.cell_costs),
and each rank's share is split into `--steps` slices of equal estimated cost
(consecutive runs of the engine's largest-n-first order, `--slices ordered`;
or LPT mixes, `--slices lpt`).  A *step* is one slice submitted to the rank's
liboi session (oi_session_*: continuous batching across calls, so later
slices' cells fill the GPU while earlier slices' slowest cells finish); step k
waits for slice k-8 (`--depth 8`), and the timed region ends when every slice
is complete and the posterior fields are on rank 0 (one gather).  Measured on
one MI355X (profiles/r02/): ordered/depth 1 57.1, ordered/depth 3 59.0,
lpt/depth 3 58.0 cells/s; one whole-day oi_gpr_batch call 61.6 (round 1).  So `--steps K` times exactly the whole day once,
whatever K; total work is fixed as N grows ("scaling": "strong").  `--warmup W`
runs W untimed slices of 24 separate small cells (n ~ U{300..1200}) through the
same session first.

Other workloads: `days` (weak scaling: every rank fits its own synthetic day,
seed + rank, in `--steps` slices), `predict` (config 2: 1000 cells x n = 500,
fixed hypers, per step), `single` (config 1: one n = 200 cell fitted per step,
one blocking call each -- a latency figure), `nystrom` / `svgp` (the
notebooks' approximate GPs).

Inputs are resident in HBM before the timed region (device-input C-ABI path).
The timed region is bracketed by barrier + device synchronise on every rank and
the max over ranks is reported.  `--budget-s` (default 420 s of wall clock
from process start) stops submitting slices early rather than being killed: the
line then says `"truncated": true` with the slices actually timed.  The CPU
baseline runs after the GPU leg (rank 0, N = 1) inside the remaining budget.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
                       [--workload day|days|season|predict|single|nystrom|svgp]
Multi-GPU: `python bench.py --gpus N` starts N rank processes itself (one per
GPU, torch.distributed over RCCL; launch_ranks below) before anything touches
the GPU, or run it under `python -m torch.distributed.run --nproc-per-node N
bench.py --gpus N` -- the same code path per rank.  --gpus must equal the
world size; more ranks than visible GPUs is refused unless OI_DIST_BACKEND=gloo
(the one-GPU rehearsal: ranks share cuda:0, collectives on the host).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

# a rank started by launch_ranks counts its --budget-s from the launcher's start
T_PROC = float(os.environ.get('OI_BENCH_T0', '') or time.time())
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6   # MI355X fp64 matrix (= vector) dense peak, spec
PEAK_HBM_GBS = 8000.0     # MI355X HBM3E peak, MI355X_MICROARCH.md
LAUNCH_GRACE_S = 600.0    # launcher: ranks may run this long past --budget-s (parity check, teardown)
METRIC = "grid-cells/sec (full GP fit+predict), 25 km pan-Arctic day, fp64"
X0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])  # GPR:217
X0_12P5 = np.array([np.log(12.5e3), np.log(12.5e3), 0.0, 0.0, 0.0, np.log(.1)])  # GPR:217, grid_res = 12.5


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--workload', default='day',
                   choices=['day', 'days', 'season', 'predict', 'single', 'nystrom', 'svgp', 'twopass'])
    p.add_argument('--season-shares', type=int, default=8,
                   help='season workload: the 12.5 km day is LPT-split into this many GPU shares; rank r '
                        'fits share r (config 5 = 8 shares on 8 GPUs; at N = 1 one 1/8 share)')
    p.add_argument('--season-days', type=int, default=1,
                   help='season workload: consecutive season days (seed + d) whose share r rank r fits, in order, '
                        'through one session (config 5 is 30 days on 8 GPUs)')
    p.add_argument('--day-shares', type=int, default=0,
                   help='day workload: LPT-split the day into this many GPU shares (default: one per rank) and fit '
                        'share --share (default: this rank\'s) -- e.g. one 8-GPU share of config 4 on one GPU')
    p.add_argument('--share', type=int, default=-1, help='day workload with --day-shares: the share to fit')
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--day-cells', type=int, default=0,
                   help='day / days: only the first K cells of the day (0: all 9997) -- quick rehearsals only')
    p.add_argument('--slices', default='ordered', choices=['lpt', 'ordered'],
                   help='day slices: equal-cost LPT mixes (lpt) or consecutive runs of the '
                        'largest-n-first order (ordered)')
    p.add_argument('--depth', type=int, default=None,
                   help='slices in flight beyond the one waited on (default: 8 for a whole day on one GPU; '
                        'every slice for a rank share of the day, config 4 -- profiles/r04/day_share_8of8.json; '
                        '8 for nystrom)')
    p.add_argument('--pregathered', action='store_true',
                   help='day / season: submit each slice from pre-gathered per-cell inputs (round 2) instead of '
                        'the radius query + gather over the pooled training set inside the timed region')
    p.add_argument('--max-pool', type=int, default=4096, help='max resident cells of the session (0: library default)')
    p.add_argument('--budget-s', type=float, default=420.0,
                   help='wall-clock budget from process start; stop submitting slices beyond it')
    p.add_argument('--nys-cells', type=int, default=0, help='nystrom workload: cells per rank-step')
    p.add_argument('--nys-oneshot', action='store_true',
                   help='nystrom workload: one blocking oi_nystrom_fit_batch call per step (round 2) instead '
                        'of a session fed one batch per step')
    p.add_argument('--svgp-cells', type=int, default=256, help='svgp workload: cells per rank-step')
    p.add_argument('--svgp-iters', type=int, default=10000, help='svgp workload: Adam steps per cell')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-prime', action='store_true',
                   help='skip the untimed priming call (profiler runs: every dispatch is then a timed one)')
    p.add_argument('--cpu-cores', type=int, default=0,
                   help='CPU baseline worker processes; 0: the host cores this process may use')
    p.add_argument('--timed-profile', default='auto', choices=['auto', 'on', 'off'],
                   help='per-launch HIP events inside the timed region (auto: on for day/days/season; off for '
                        'single/predict, whose roofline then comes from a second, profiled pass)')
    p.add_argument('--parity-cells', type=int, default=24,
                   help='day workloads: timed cells re-checked against the CPU oracle at the GPU fit\'s '
                        'hypers (T1, SURVEY §8c), stratified over n; 0 = skip')
    p.add_argument('--twopass-small', action='store_true',
                   help='twopass workload: a small binned day (48 x 48 grid, ~100 cells) -- tests / rehearsals only')
    p.add_argument('--dump', default='', help='write per-cell n, m, evals, status of the timed cells (.npz)')
    p.add_argument('--out', default='')
    return p.parse_args()


def elapsed():
    return time.time() - T_PROC


def log(msg):
    print(f"[bench {elapsed():6.1f}s] {msg}", file=sys.stderr, flush=True)


# ----------------------------------------------------------------- host cores
def host_cores(args=None):
    """-> (workers, description).  The CPUs this process may run on: the
    smaller of sched_getaffinity and the cgroup CPU quota (cpu.max).  On the
    GPU box affinity lists the whole machine (256) while the quota is 16 CPUs,
    so more workers than the quota would only time-share those 16."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = int(q) / int(per)
    except Exception:
        pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    if args is not None and args.cpu_cores:
        n = args.cpu_cores
    desc = f"sched_getaffinity {aff} CPUs, cgroup cpu.max quota {quota if quota is not None else 'none'}"
    return n, desc


# ----------------------------------------------------------------- workloads
def split_slices(sizes, k, how='lpt', sites=None):
    """Cell index sets of ``k`` slices of equal estimated cost (driver.cell_costs)."""
    from optimalinterpolation_amd import driver
    k = max(1, min(int(k), len(sizes))) if len(sizes) else 1
    costs = driver.cell_costs(sizes, sites=sites)
    if how == 'lpt':
        return driver.lpt_partition(costs, k)
    order = np.argsort(-np.asarray(sizes), kind='stable')  # the engine's admission order
    cum = np.cumsum(costs[order])
    cut = np.searchsorted(cum, cum[-1] * np.arange(1, k) / k)
    return [np.sort(p) for p in np.split(order, cut)]


POOL_PITCH_M = 1.0e6  # lattice pitch of the pooled training set (> 2 x (RADIUS_M + grid spacing))


def pool_training_set(slices, grid_m, torch, dev):
    """All timed cells as ONE training set resident in HBM, so that the radius
    query and the gather of GPR:159-161 (oi_ball_query / oi_gather_rows) run
    inside the timed region like the rest of GPR3D.  The synthetic day draws
    each cell's observations on their own (n ~ U{300..3000}), so
    the points the query searches are the observations translated cell by
    cell -- cell g's centre onto node g of a 1000 km lattice, every one of its
    observations by the same amount -- and no ball of radius RADIUS_M + grid_m
    reaches another cell's points: the query returns exactly the cell's
    observations in their original order.  The gathered columns are the
    observations as drawn, so the fit sees bit-identical inputs (the Matérn
    distances are formed from sqrt(3) x / ell, GPR:93, which is not exactly
    translation invariant)."""
    from optimalinterpolation_amd import synthetic
    cols, sx, sy, q_all, g = [[], [], [], []], [], [], [], 0
    for cells in slices:
        q = np.empty((cells.ncell, 2))
        for c in range(cells.ncell):
            lx, ly = POOL_PITCH_M * (1 + g % 128), POOL_PITCH_M * (1 + g // 128)
            a, b = cells.offs[c], cells.offs[c + 1]
            x = cells.xyt[a:b]
            for d in range(3):
                cols[d].append(x[:, d])
            cols[3].append(cells.z[a:b])
            sx.append(x[:, 0] - cells.xs[c, 0] + lx)
            sy.append(x[:, 1] - cells.xs[c, 1] + ly)
            q[c] = lx, ly
            g += 1
        q_all.append(torch.from_numpy(q).to(dev))
    cat = [np.concatenate(cc) if cc else np.zeros(0) for cc in cols]
    dcols = tuple(torch.from_numpy(cc).to(dev).contiguous() for cc in cat)
    pts = np.column_stack([np.concatenate(sx), np.concatenate(sy)]) if sx else np.zeros((0, 2))
    return {"cols": dcols, "pts": torch.from_numpy(np.ascontiguousarray(pts)).to(dev), "q": q_all,
            "r": synthetic.RADIUS_M + grid_m, "M": int(len(cat[0]))}


def check_shares(args, world, shares):
    """--day-shares / --share: a share run fits one share on one
    GPU; with N ranks the day is split N ways and rank r fits share r."""
    if args.share >= 0 and world > 1:
        raise SystemExit("bench.py: --share picks the share of a one-GPU run; with N ranks rank r fits share r")
    if args.share >= 0 and not args.day_shares:
        raise SystemExit("bench.py: --share needs --day-shares")
    if args.share >= shares:
        raise SystemExit(f"bench.py: --share {args.share} but only {shares} shares")
    if world > 1 and args.day_shares not in (0, world):
        raise SystemExit(f"bench.py: --day-shares {args.day_shares} with {world} ranks would leave shares unfitted")


def default_depth(args, world, nslices, per_day=None):
    """Slices in flight beyond the one waited on, keyed on the per-rank work
    (ADVICE r4), never on the GPU count alone:
      * a rank's SHARE of a day (config 4 at N > 1, --day-shares runs, and the
        season, whose every rank -- N = 1 included -- fits one 1/8 share) goes
        into its session at once, so the rounds stay near the 1-GPU resident
        size (8 shares at depth 20 on one GPU: 0.90 projected efficiency,
        profiles/r04/day_share_8of8.json);
      * the season's depth is keyed on the slices of ONE day (``per_day``,
        ADVICE r5), so consecutive days stream through the session instead of
        all K days' inputs being submitted at once;
      * a WHOLE day per rank (config 3, and `days` at any N) keeps 8 slices
        in flight, as the headline always has."""
    if args.workload == 'season' and per_day:
        return max(1, int(max(per_day))), "the slices of one season day (a rank's share of that day)"
    share = args.workload == 'season' or (args.workload == 'day' and (world > 1 or args.day_shares))
    return (max(1, nslices), "every slice (a rank's share of a day)") if share else (8, "8 (a whole day per rank)")


def build_slices(args, rank, world):
    """-> (timed slices of this rank, warmup slices, opt, config, scaling,
    cells per rank of every rank)."""
    from optimalinterpolation_amd import driver, synthetic
    warm = [synthetic.make_cells(np.random.default_rng(900 + g).integers(300, 1201, 24),
                                 seed=1000 + 97 * g + rank) for g in range(args.warmup)]
    if args.workload == 'season':
        # config 5: rank r fits share r of each of --season-days consecutive
        # season days (seed + d), the days one after another through one
        # session; each day's share in ~steps/K slices of equal estimated cost
        shares = max(int(args.season_shares), world)
        K = max(1, int(args.season_days))
        per_day = [args.steps // K + (1 if d < args.steps % K else 0) for d in range(K)]
        out, ncell_day, tot, mine_n, counts = [], 0, 0, 0, [0] * world
        for d in range(K):
            cen, sizes = synthetic.season_day_plan(seed=args.seed + d)
            est = driver.expected_sites(sizes, grid_m=synthetic.GRID_12P5_M)
            parts = driver.lpt_partition(driver.cell_costs(sizes, sites=est), shares)
            mine = synthetic.season_cells(cen, sizes, parts[rank], seed=args.seed + d)
            sl = split_slices(mine.sizes, max(1, per_day[d]), args.slices, driver.site_counts(mine))
            out += [mine.subset(s) for s in sl]
            ncell_day = len(sizes)
            tot += int(sum(len(parts[r]) for r in range(world)))
            mine_n += int(mine.ncell)
            for r in range(world):
                counts[r] += len(parts[r])
        days = "one day" if K == 1 else f"{K} consecutive days (seeds {args.seed}..{args.seed + K - 1})"
        cfg = {"workload": (f"config 5: {days} of the 12.5 km season (640x640 grid, {ncell_day} cells a day, "
                            f"n ~ U{{300..5000}}), opt=True fit+predict; each day LPT-split into {shares} GPU "
                            f"shares, this run fits {world} of them (share r on rank r), the days in order through "
                            f"one session, one slice per step"),
               "day_cells": int(ncell_day), "season_days": K, "n_obs_per_cell": "U{300..5000}", "grid_km": 12.5,
               "x0": "GPR_CS2S3.py:217 with grid_res = 12.5", "shares": shares, "slices_per_day": per_day,
               "cells_total": tot, "cells_per_rank": mine_n,
               "parallelism": f"dp{world} ({shares}-way LPT partition on E(n) m^3, m = expected sites)"}
        return out, warm, True, cfg, "weak", counts
    if args.workload in ('day', 'days'):
        seed = args.seed + (rank if args.workload == 'days' else 0)
        day = synthetic.make_day(seed=seed, max_cells=args.day_cells or None)
        common = {"day_cells": int(day.ncell), **({"day_cells_limit": args.day_cells} if args.day_cells else {}), "n_obs_per_cell": "U{300..3000}", "grid_km": 25,
                  "x0": "GPR_CS2S3.py:217", "slices": args.slices}
        day_sites = driver.site_counts(day)
        if args.workload == 'day':
            shares = max(int(args.day_shares), world)
            check_shares(args, world, shares)
            parts = driver.lpt_partition(driver.cell_costs(day.sizes, sites=day_sites), shares)
            idx = [args.share if args.share >= 0 else r for r in range(world)]
            mine = day.subset(parts[idx[rank]])
            mine_sites = day_sites[parts[idx[rank]]]
            if shares == world:
                cfg = {"workload": ("25km pan-Arctic day, opt=True fit+predict per cell "
                                    f"(config {'3' if world == 1 else '4'}: the whole day on {world} GPU"
                                    f"{'s' if world > 1 else ''}, one slice per step)"),
                       **common, "cells_total": int(day.ncell), "cells_per_rank": int(mine.ncell),
                       "parallelism": f"dp{world} (LPT cell partition on E(n) m^3, one RCCL gather)"}
            else:
                cfg = {"workload": (f"config 4 share: the 25km day LPT-split into {shares} GPU shares, this run "
                                    f"fits share(s) {idx} ({world} GPU), one slice per step"),
                       **common, "day_cells_total": int(day.ncell),
                       "cells_total": int(sum(len(parts[i]) for i in idx)), "cells_per_rank": int(mine.ncell),
                       "shares": shares, "share": idx[rank],
                       "parallelism": f"{shares}-way LPT partition on E(n) m^3; {world} of them here"}
            scaling = "strong"
            counts_all = [len(parts[i]) for i in idx]
        else:
            mine, mine_sites = day, day_sites
            cfg = {"workload": "one synthetic 25km day per rank (seed + rank), opt=True fit+predict, "
                               "one slice per step", **common, "cells_total": int(day.ncell) * world,
                   "parallelism": f"dp{world} (a day per GPU, one RCCL gather)"}
            scaling = "weak"
            counts_all = [int(day.ncell)] * world  # day_centres() is the same grid for every seed
        sl = split_slices(mine.sizes, args.steps, args.slices, mine_sites)
        return [mine.subset(s) for s in sl], warm, True, cfg, scaling, counts_all
    if args.workload == 'predict':
        cells = [synthetic.make_cells([500] * 1000, seed=args.seed + 7919 * k + rank) for k in range(args.steps)]
        cfg = {"workload": "config 2: 1000 cells x n=500, fixed hypers (predict-only), per step",
               "cells_per_step": 1000, "parallelism": f"dp{world}"}
        warm = [synthetic.make_cells([500] * 100, seed=5000 + g) for g in range(args.warmup)]
        return cells, warm, False, cfg, "weak", [1000 * args.steps] * world
    cells = [synthetic.make_cells([200], seed=args.seed + 31 * k + rank) for k in range(args.steps)]
    cfg = {"workload": "config 1: single cell, n=200, opt=True, one blocking call per step",
           "cells_per_step": 1, "parallelism": f"dp{world}"}
    warm = [synthetic.make_cells([200], seed=7000 + g) for g in range(args.warmup)]
    return cells, warm, True, cfg, "weak", [args.steps] * world


# ----------------------------------------------------------------- cpu baseline
CPU_JOB = r'''
import json, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import gp_oracle as O
from optimalinterpolation_amd import synthetic
kind, n, seed = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cells = synthetic.make_cells([n], seed=seed)
x, y, xs = cells.cell(0)
mX = np.ones(n) * cells.mean
if kind == 'eval':
    h = np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), np.log(.1)])
    te, tp = [], []
    for _ in range(2):  # the second call is the warm one (the first touches fresh pages)
        t = time.perf_counter(); O.neg_log_ml(h, x, y, mX); te.append(time.perf_counter() - t)
        t = time.perf_counter(); O.predict(x, y, xs, cells.mean, np.exp(h[:3]), np.exp(h[3]), np.exp(h[4]))
        tp.append(time.perf_counter() - t)
    te, tp = te[-1], tp[-1]
    print(json.dumps({"kind": kind, "n": n, "seed": seed, "eval_s": te, "pred_s": tp}))
else:
    trace = []
    t = time.perf_counter()
    O.gp_cell(x, y, xs[0], cells.mean, opt=True, x0=O.X0_PRODUCTION, trace=trace)
    print(json.dumps({"kind": kind, "n": n, "seed": seed, "fit_s": time.perf_counter() - t,
                      "evals": len(trace)}))
'''

EVAL_PROBES = (300, 600, 1000, 1500, 2000, 2500, 3000)
FIT_SAMPLE = tuple(range(300, 601, 20))   # 16 cells, stratified over n in [300, 600]
FIT_LARGE = (2000, 2000, 1500, 1500)      # k at large n (k from small fits alone over-predicted
                                          # n = 1500..3000 fits by 4-16 %, profiles/r06/cpu_model_check.json)


def run_jobs(jobs, workers, deadline):
    """Run oracle jobs [(kind, n, seed)], ``workers`` single-threaded-BLAS
    processes at a time (one MPI rank per core in the reference); jobs not
    started before ``deadline`` (time.time()) are skipped."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    pending, running, res = list(jobs), [], []
    while pending or running:
        while pending and len(running) < workers and time.time() < deadline:
            kind, n, seed = pending.pop(0)
            running.append(subprocess.Popen([sys.executable, '-c', CPU_JOB, ROOT, kind, str(n), str(seed)],
                                            stdout=subprocess.PIPE, text=True, env=env))
        if pending and time.time() >= deadline:
            pending = []
        for p in list(running):
            if p.poll() is not None:
                out = p.stdout.read()
                running.remove(p)
                if p.returncode == 0 and out.strip():
                    res.append(json.loads(out.strip().splitlines()[-1]))
        time.sleep(0.05)
    return res


def reference_evals_model():
    """E(n): the REFERENCE's own SMLII evaluations per GPR3D(opt=True) fit.

    Source: tests/golden/day_ref_fits.npz -- GPR_CS2S3.py:143-191 run on the
    fixture's cells of the bench day itself (synthetic.make_day(seed=0)) in 5
    observation orders each (tests/golden/make_day_fits.py): the mean over the
    fixture's cells and runs in each 300-wide n bucket from 300 to 3000.  Above
    n = 3000 (config 5) the reference's fits of n = 2500..5000 in
    tests/golden/fit_large.npz, fitted a + b n.  -> (E(n) callable, description)."""
    d = np.load(os.path.join(ROOT, 'tests', 'golden', 'day_ref_fits.npz'))
    sizes, ev = d['sizes'], d['evals'].astype(float)
    edges = np.arange(300, 3001, 300)
    bucket = np.array([ev[(sizes >= lo) & (sizes < (lo + 300 if lo < 2700 else 3001))].mean() for lo in edges[:-1]])
    fx = np.load(os.path.join(ROOT, 'tests', 'golden', 'fit_large.npz'))
    m = fx['sizes'] >= 2500
    en = np.repeat(fx['sizes'][m], fx['evals'].shape[1]).astype(float)
    big, *_ = np.linalg.lstsq(np.stack([np.ones_like(en), en], 1), fx['evals'][m].ravel().astype(float), rcond=None)

    def E(n):
        n = np.asarray(n, float)
        k = np.clip(((n - 300) // 300).astype(int), 0, len(bucket) - 1)
        return np.where(n > 3000, big[0] + big[1] * n, bucket[k])
    desc = (f"the reference's own evaluations per fit: per 300-wide n bucket the mean of its "
            f"{ev.size} fits of {len(sizes)} cells of this day (tests/golden/day_ref_fits.npz: "
            + ", ".join(f"{lo}: {b:.1f}" for lo, b in zip(edges[:-1], bucket))
            + f"); n > 3000: {big[0]:.1f} + {big[1]:.4f} n from tests/golden/fit_large.npz")
    # the fixture's mean reweighted to the day's n distribution (uniform on 300..3000)
    return E, desc, float(np.mean(bucket))


def cpu_baseline(sizes, gpu_evals, workers, cores_desc, deadline, extra_pred=0):
    """The CPU oracle (oracle/gp_oracle.py, bit-exact restatement of
    GPR_CS2S3.py:78-191 with scipy's CG) on this host's cores, one
    single-threaded-BLAS process per core:
      * t_eval(n), t_pred(n): one SMLII evaluation and one predict block at
        n = 300..3000 (the second of two calls in the process), 3 repetitions
        each (median), all timed while ``workers`` processes run at once,
        fitted t = a + b n^2 + c n^3 by relative least squares;
      * k(n): the ratio measured / modelled time of full oracle GPR3D(opt=True)
        fits run on the same host, each modelled as its own evaluation count x
        t_eval(n) + t_pred(n) (k absorbs the optimiser's Python per evaluation,
        which matters at small n): the median over 16 fits at n = 300..600
        (k_small) and over 4 fits at n = 1500..2000 (k_large), interpolated in
        log t_eval(n) between the two groups' median sizes and held constant
        outside them; the residual of every fit after k(n) is reported;
      * E(n): the reference's own evaluations per cell on this day's cells
        (reference_evals_model: tests/golden/day_ref_fits.npz), not the GPU's;
      * value = cells / (sum over the timed cells of k(n) E(n) t_eval(n) + t_pred(n))
        x workers -- extrapolated, labelled so."""
    t0 = time.time()
    jobs = [('eval', n, 11 * n + r) for n in sorted(EVAL_PROBES, reverse=True) for r in range(3)]
    # the large fits first (each runs ~0.5-2 minutes), then the probes and the small fits
    jobs = ([('fit', n, 13 * n + 1 + r) for r, n in enumerate(FIT_LARGE)] + jobs[:6]
            + [('fit', n, 13 * n + 1) for n in FIT_SAMPLE] + jobs[6:])
    res = run_jobs(jobs, workers, deadline)
    ev = [r for r in res if r['kind'] == 'eval']
    fits = [r for r in res if r['kind'] == 'fit']
    if len({r['n'] for r in ev}) < 3 or not fits:
        raise RuntimeError(f"CPU baseline incomplete before the budget: {len(ev)} probes, {len(fits)} fits")
    ns = sorted({r['n'] for r in ev})
    med = {n: (float(np.median([r['eval_s'] for r in ev if r['n'] == n])),
               float(np.median([r['pred_s'] for r in ev if r['n'] == n]))) for n in ns}
    na = np.array(ns, float)
    A = np.stack([np.ones_like(na), na ** 2, na ** 3], 1)

    def rel_lstsq(y):  # minimise the RELATIVE residual: small n is not swamped by n = 3000
        y = np.asarray(y, float)
        c, *_ = np.linalg.lstsq(A / y[:, None], np.ones_like(y), rcond=None)
        return c
    ce = rel_lstsq([med[n][0] for n in ns])
    cp = rel_lstsq([med[n][1] for n in ns])

    def t_eval(n):
        return ce[0] + ce[1] * n ** 2 + ce[2] * n ** 3

    def t_pred(n):
        return cp[0] + cp[1] * n ** 2 + cp[2] * n ** 3

    n = np.asarray(sizes, float)
    gpu_evals = np.asarray(gpu_evals, float)
    model = np.array([f['evals'] * t_eval(f['n']) + t_pred(f['n']) for f in fits])
    meas = np.array([f['fit_s'] for f in fits])
    fn = np.array([f['n'] for f in fits], float)
    sm_f, lg_f = fn <= 600, fn > 600
    k_s = float(np.median((meas / model)[sm_f])) if sm_f.any() else float(np.median(meas / model))
    k_l = float(np.median((meas / model)[lg_f])) if lg_f.any() else k_s
    n_s = float(np.median(fn[sm_f])) if sm_f.any() else 450.0
    n_l = float(np.median(fn[lg_f])) if lg_f.any() else n_s

    def k_of(nn):  # linear in log t_eval between the two calibration groups, constant outside
        x = np.log(t_eval(np.asarray(nn, float)))
        xs, xl = np.log(t_eval(n_s)), np.log(t_eval(n_l))
        w = np.clip((x - xs) / (xl - xs), 0.0, 1.0) if xl > xs else np.zeros_like(x)
        return k_s + w * (k_l - k_s)
    k = float(k_of(np.median(sizes))) if len(sizes) else k_s
    resid = meas / (k_of(fn) * model) - 1.0
    try:
        E, e_src, e_fix = reference_evals_model()
        e_cells = E(n)
    except Exception as e:  # fixture missing: the sample fits' mean, flat in n
        e_cells = np.full(len(n), float(np.mean([f['evals'] for f in fits])))
        e_src, e_fix = f"the {len(fits)} sample fits' mean evaluation count, flat in n ({e!r})", None
    t_cells = k_of(n) * e_cells * t_eval(n) + (1 + extra_pred) * t_pred(n)  # extra_pred: pass 2 (GPR:316-319)
    value = len(n) / (float(np.sum(t_cells)) / workers)
    small = n <= 600
    return {"value": value, "unit": "grid-cells/s", "cores": workers, "kind": "port",
            "sample": (f"oracle/gp_oracle.py (bit-exact restatement of GPR_CS2S3.py:78-191 + scipy CG) on "
                       f"{workers} single-threaded-BLAS processes ({cores_desc}); measured: one SMLII eval + "
                       f"one predict at n={ns} x3 reps (median, fitted a+bn^2+cn^3, relative least squares) and "
                       f"{int(sm_f.sum())} full GPR3D(opt=True) fits at n=300..600 and {int(lg_f.sum())} at "
                       f"n=1500..2000 (measured / modelled time k = {k_s:.3f} at n={n_s:.0f}, {k_l:.3f} at "
                       f"n={n_l:.0f}, interpolated in log t_eval; residuals after k(n) {np.min(resid):+.3f} .. "
                       f"{np.max(resid):+.3f}); "
                       f"extrapolated to the {len(n)} timed cells with E(n) = {e_src} "
                       f"({time.time() - t0:.0f} s wall): extrapolated"),
            "e_cpu_mean_timed_cells": round(float(np.mean(e_cells)), 2),
            "e_ref_fixture_mean_day_weighted": round(e_fix, 2) if e_fix is not None else None,
            "e_gpu_mean_timed_cells": round(float(np.mean(gpu_evals)), 2),
            "e_cpu_sample_fits": round(float(np.mean([f['evals'] for f in fits])), 2),
            "e_gpu_small": round(float(np.mean(gpu_evals[small])), 2) if small.any() else None,
            "fit_time_model_k": round(k, 4),
            "fit_time_model_k_small_large": [round(k_s, 4), round(k_l, 4)],
            "fit_time_model_k_anchor_n": [n_s, n_l],
            "fit_sizes": [int(v) for v in fn],
            "fit_time_residual_max_abs": round(float(np.max(np.abs(resid))), 4),
            "fit_time_total_residual": round(float(np.sum(k * model) / np.sum(meas) - 1.0), 4),
            "fit_time_residuals": [round(float(r), 4) for r in resid],
            "probe_s": {str(kk): [round(v[0], 5), round(v[1], 5)] for kk, v in med.items()},
            "t_eval_coef": [float(v) for v in ce], "t_pred_coef": [float(v) for v in cp],
            "cpu_s_per_cell_mean": round(float(np.mean(t_cells)), 3)}


# ----------------------------------------------------------------- nystrom
NYS_N, NYS_M, NYS_CELLS = 4600, 925, 32

NYS_PROBE = r'''
import os, sys, time, json
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import nystrom_oracle as N
from optimalinterpolation_amd import synthetic
n, M = int(sys.argv[2]), int(sys.argv[3])
cells = synthetic.make_cells([n], seed=77)
x, z, xs = cells.cell(0)
y = z - cells.mean
h = np.log([2.5e4, 2.5e4, 1.0, 1.0, 0.1])
t = time.perf_counter(); N.neg_log_ml(h, x, y, M); te = time.perf_counter() - t
t = time.perf_counter(); N.predict(x, y, xs, list(np.exp(h[:3])), np.exp(h[3]), np.exp(h[4]), cells.mean, M)
tp = time.perf_counter() - t
print(json.dumps({"n": n, "M": M, "eval_s": te, "pred_s": tp}))
'''


def nystrom_cpu_baseline(evals, cores):
    """The oracle (NB1 restated, bit-exact vs the notebook's functions) timed
    for one SMLII(approx=True) evaluation + one GPR(approx=True) at n=4600,
    M=925 with single-threaded OpenBLAS, scaled by the GPU run's measured
    objective evaluations per cell, ``cores`` such processes in parallel."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    t0 = time.time()
    out = subprocess.run([sys.executable, '-c', NYS_PROBE, ROOT, str(NYS_N), str(NYS_M)],
                         capture_output=True, text=True, env=env, timeout=600, check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    t_cell = float(np.mean(evals)) * r['eval_s'] + r['pred_s']
    return {"value": cores / t_cell, "unit": "grid-cells/s", "cores": cores, "kind": "port",
            "sample": (f"oracle/nystrom_oracle.py (bit-exact vs GP_example.ipynb's Nystroem/SMLII/GPR) "
                       f"timed for 1 SMLII(approx) eval ({r['eval_s']:.2f} s) + 1 GPR(approx) "
                       f"({r['pred_s']:.2f} s) at n={NYS_N}, M={NYS_M}, 1 OpenBLAS thread "
                       f"({time.time() - t0:.0f} s wall); x {float(np.mean(evals)):.1f} measured "
                       f"evals/cell, {cores} such processes in parallel: extrapolated"),
            "probe": r}


def main_nystrom(args, torch, dist, world, rank, gpu, cdev):
    from optimalinterpolation_amd import _lib, nystrom, synthetic
    dev = torch.device('cuda', gpu)
    x0 = nystrom.default_x0()
    ncell = args.nys_cells or NYS_CELLS
    steps = []
    for k in range(args.warmup + args.steps):
        cells = synthetic.make_cells([NYS_N] * ncell, seed=args.seed + 1000 * rank + k)
        sel, soffs = nystrom._ragged_sel(cells.offs, NYS_M)
        y = cells.z - cells.mean  # NB1 passes outputs - mX
        steps.append((cells, sel, soffs, torch.from_numpy(cells.xyt).to(dev).contiguous(),
                      torch.from_numpy(y).to(dev).contiguous()))
    torch.cuda.synchronize()

    def run(k, profile):
        cells, sel, soffs, xd, yd = steps[k]
        return _lib.nystrom_fit_batch(xd, yd, cells.offs, sel, soffs, x0, cells.xs, cells.mean,
                                      device=gpu, device_inputs=True, profile=profile)

    def run_session(ks):  # one batch per step through a session: step k waits for step k - depth
        outs, tickets = {}, {}
        with _lib.NystromSession(device=gpu, device_inputs=True, profile=True) as sess:
            for i, k in enumerate(ks):
                cells, sel, soffs, xd, yd = steps[k]
                tickets[k] = sess.submit(xd, yd, cells.offs, sel, soffs, x0, cells.xs, cells.mean)
                if i >= args.depth:
                    kk = ks[i - args.depth]
                    outs[kk] = sess.wait(tickets[kk])
            for k in ks:
                if k not in outs:
                    outs[k] = sess.wait(tickets[k])
        return [outs[k] for k in ks]

    if not args.no_prime:  # library / code-object initialisation, not a step
        pc = synthetic.make_cells([300], seed=4321)
        ps, po = nystrom._ragged_sel(pc.offs, 60)
        _lib.nystrom_fit_batch(pc.xyt, pc.z - pc.mean, pc.offs, ps, po, x0, pc.xs, pc.mean, device=gpu)
    for k in range(args.warmup):
        run(k, False)
    _lib.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.nys_oneshot:
        outs = [run(k, True) for k in range(args.warmup, args.warmup + args.steps)]
    else:
        outs = run_session(list(range(args.warmup, args.warmup + args.steps)))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ncells = ncell * args.steps * world
    info = np.concatenate([o[2] for o in outs])
    evals = info[:, 3].astype(float)
    kern = {k: v for k, v in _lib.profile_json()['kernels'].items() if k.startswith('nys_')}
    dom = max(kern, key=lambda k: kern[k]['total_ms'])
    kd = kern[dom]
    sec = kd['total_ms'] / 1e3
    if kd['flops'] > 0 and (kd['bytes'] == 0 or kd['flops'] / kd['bytes'] > 10):
        ach, peak, unit, bound = kd['flops'] / sec / 1e12, PEAK_FP64_TFLOPS, "TFLOP/s", "mfma"
    else:
        ach, peak, unit, bound = kd['bytes'] / sec / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
    roofline = {"bound": bound, "kernel": dom, "achieved": round(ach, 3), "peak": peak, "unit": unit,
                "frac": round(ach / peak, 4), "traffic": None,
                "launches": kd['launches'], "avg_launch_ms": kd['total_ms'] / max(kd['launches'], 1),
                "flops_per_launch": kd['flops'] / max(kd['launches'], 1),
                "bytes_per_launch": kd['bytes'] / max(kd['launches'], 1),
                "stages_ms": {k: round(v['total_ms'], 3) for k, v in kern.items()},
                "stage_model": "per-cell stage of oi_nystrom.hip timed with HIP events; algorithmic "
                               "flops (Ki GEMM 2 n^2 M, eigh 4 M^3 ...) / bytes (objective pass 8 n^2)"}
    line = {"metric": "grid-cells/sec (Nystrom fit+predict, NB1 cell 5), fp64",
            "value": round(ncells / dt, 4), "unit": "grid-cells/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded cells of the SURVEY §8d generator)",
            "config": {"workload": f"Nystrom (GP_example.ipynb cell 5): {ncell} cells x n={NYS_N}, "
                                   f"M={NYS_M} per rank per step, CG fit + predict"
                                   + (", one blocking call per step" if args.nys_oneshot else
                                      f", one batch per step through a fit session (depth {args.depth})"),
                       "cells_per_step": ncell * world},
            "evals_per_cell": round(float(np.mean(evals)), 2), "roofline": roofline, **args.dist_fields}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = host_cores(args)[0]
        try:
            line["cpu_baseline"] = nystrom_cpu_baseline(evals, cores)
        except Exception as e:
            line["cpu_baseline"] = {"value": None, "error": repr(e)}
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, 'w') as f:
                f.write(s + '\n')
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------- svgp
SVGP_N, SVGP_M, SVGP_B = 4600, 50, 100
SVGP_INIT = [25e3, 25e3, 1.0, 1.0, 0.1]  # NB2: lengthscales, kernel variance, noise variance

SVGP_PROBE = r'''
import os, sys, time, json
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import svgp_oracle as O
from optimalinterpolation_amd import synthetic
n, M, B, steps = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
cells = synthetic.make_cells([n], seed=91)
x, z, xs = cells.cell(0)
t = time.perf_counter()
p, log = O.train(x, z, O.notebook_Z(x, M), [25e3, 25e3, 1.0], 1.0, 0.1, cells.mean, B=B, iterations=steps, seed=1)
O.predict_f(p, xs)
print(json.dumps({"steps": steps, "s": time.perf_counter() - t}))
'''


def svgp_cpu_baseline(iters, cores):
    """The oracle (GPflow SVGP + TF2 Adam restated in NumPy) timed for 300 Adam
    steps of one cell with single-threaded OpenBLAS, scaled to the workload's
    steps, ``cores`` such processes in parallel."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1")
    steps = 300
    out = subprocess.run([sys.executable, '-c', SVGP_PROBE, ROOT, str(SVGP_N), str(SVGP_M), str(SVGP_B),
                          str(steps)], capture_output=True, text=True, env=env, timeout=600,
                         check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    t_cell = r['s'] / steps * iters * 1.1  # + the notebook's logging pass every 10 steps
    return {"value": cores / t_cell, "unit": "grid-cells/s", "cores": cores, "kind": "port",
            "sample": (f"oracle/svgp_oracle.py (GPflow SVGP + TF2 Adam restated) timed for {steps} Adam "
                       f"steps of one n={SVGP_N}, M={SVGP_M}, B={SVGP_B} cell ({r['s']:.2f} s, 1 OpenBLAS "
                       f"thread), scaled to {iters} steps + 10% logging passes, {cores} such processes "
                       f"in parallel: extrapolated"), "probe": r}


def main_svgp(args, torch, dist, world, rank, gpu, cdev):
    from optimalinterpolation_amd import _lib, svgp, synthetic
    dev = torch.device('cuda', gpu)
    k, iters = args.svgp_cells, args.svgp_iters
    steps = []
    for s in range(args.warmup + args.steps):
        cells = synthetic.make_cells([SVGP_N] * k, seed=args.seed + 1000 * rank + s)
        Z = np.stack([svgp.notebook_Z(cells.cell(c)[0], SVGP_M) for c in range(k)])
        init = np.tile(SVGP_INIT + [cells.mean], (k, 1))
        steps.append((cells, Z, init, torch.from_numpy(cells.xyt).to(dev).contiguous(),
                      torch.from_numpy(cells.z).to(dev).contiguous()))
    torch.cuda.synchronize()

    def run(s):
        cells, Z, init, xd, zd = steps[s]
        return _lib.svgp_batch(xd, zd, cells.offs, Z, init, cells.xs, batch=SVGP_B, iterations=iters,
                               log_every=10, seed=s, device=gpu, device_inputs=True, profile=True)

    if not args.no_prime:
        pc = synthetic.make_cells([300], seed=4321)
        _lib.svgp_batch(pc.xyt, pc.z, pc.offs, svgp.notebook_Z(pc.xyt, 8)[None], [SVGP_INIT + [pc.mean]],
                        pc.xs, batch=50, iterations=3, device=gpu)
    for s in range(args.warmup):
        run(s)
    _lib.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [run(s) for s in range(args.warmup, args.warmup + args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ncells = k * args.steps * world
    bad = int(sum(int(o[1].sum()) for o in outs))
    kd = _lib.profile_json()['kernels']['k_svgp_train']  # HIP events around the launch
    kern_ms = kd['total_ms'] / max(kd['launches'], 1)
    ach = kd['flops'] / (kd['total_ms'] / 1e3) / 1e12
    traffic = None
    tfile = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tfile) and k == 256 and iters == 10000:  # measured for the default shape
        traffic = json.load(open(tfile)).get('k_svgp_train', {}).get('hbm_bytes_per_launch')
    roofline = {"bound": "mfma", "kernel": "k_svgp_train", "achieved": round(ach, 4),
                "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_FP64_TFLOPS, 5),
                "traffic": traffic,
                "traffic_note": ("HBM bytes per launch, rocprofv3 PMC FETCH_SIZE(x2)+WRITE_SIZE, "
                                 "profiles/r01/pmc_hbm_bytes_svgp.json: parameters / Adam moments / "
                                 "K_uf panels re-read from L2 misses, ~3.5 % of HBM bandwidth")
                if traffic else None,
                "launches": kd['launches'], "avg_launch_ms": round(kern_ms, 3),
                "flops_per_launch": kd['flops'] / max(kd['launches'], 1),
                "flop_model": "per Adam step 9 M^2 B + 10/3 M^3 (M=50, B=100) x (steps + logging/3) x cells",
                "note": "latency-bound per-cell dependency chains (one workgroup per cell); frac is "
                        "against the fp64 dense peak"}
    line = {"metric": "grid-cells/sec (SVGP fit+predict, NB2 cell 5), fp64",
            "value": round(ncells / dt, 4), "unit": "grid-cells/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded cells of the SURVEY §8d generator)",
            "config": {"workload": f"SVGP (dev/sparseGP_example.ipynb cell 5): {k} cells x n={SVGP_N}, "
                                   f"M={SVGP_M}, B={SVGP_B}, {iters} Adam steps per rank per step",
                       "cells_per_step": k * world},
            "failed_cells": bad, "roofline": roofline, **args.dist_fields}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = host_cores(args)[0]
        try:
            line["cpu_baseline"] = svgp_cpu_baseline(iters, cores)
        except Exception as e:
            line["cpu_baseline"] = {"value": None, "error": repr(e)}
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, 'w') as f:
                f.write(s + '\n')
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------- twopass
TWOPASS_CHECK = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from scipy.spatial import cKDTree
from oracle import day_oracle as D, gp_oracle as G
d = np.load(sys.argv[2])
sat, sie, x, y, mean, T, rad = d['sat'], d['sie'], d['x'], d['y'], float(d['mean']), int(d['T']), float(d['radius'])
x_train, y_train, t_train, z = D.training_set(sat, x, y)
IDs = np.where(~np.isnan(sie))
X = np.array([x[IDs], y[IDs]]).T
out = {}
if sys.argv[3] == 'smooth':   # GPR:299-307 on the GPU's own pass-1 fields: bit-exact expected
    same = []
    for k, (key, vmax) in enumerate(zip(D.SMOOTH_VMAX_KEYS, D.smooth_vmax(rad, T))):
        ref = D.smooth(d['p1'][k], vmax, sie, int(d['std']))
        a = d['sm'][k]
        same.append(bool(np.array_equal(np.isnan(a), np.isnan(ref)) and np.array_equal(a[~np.isnan(a)], ref[~np.isnan(ref)])))
    out = {"smooth_bit_exact": same}
else:                        # pass 2 (GPR:316-319 -> GPR3D opt=False, GPR:169-182) of sampled cells
    tree = cKDTree(np.array([x_train, y_train]).T)
    rel = lambda a, b: abs(a - b) / max(1.0, abs(b))
    wf, ws, ns = 0.0, 0.0, []
    for q, c in enumerate(d['cells']):
        ID = tree.query_ball_point(x=X[c, :], r=rad * 1000)
        inputs = np.array([x_train[ID], y_train[ID], t_train[ID]]).T
        hyp = tuple(float(v) for v in d['hyp'][q])
        fs, sd = G.gp_cell(inputs, z[ID], np.array([X[c, 0], X[c, 1], T // 2]), mean, opt=False, hyp=hyp)
        wf, ws = max(wf, rel(d['fs'][q], fs)), max(ws, rel(d['sd'][q], sd))
        ns.append(len(ID))
    out = {"max_rel_fs": wf, "max_rel_sd": ws, "n": ns}
print(json.dumps(out))
'''


def main_twopass(args, torch, dist, world, rank, gpu, cdev):
    """The reference's WHOLE two-pass day: GPR_CS2S3.py
    :223-246 training set, :159 radius query, :258-262 pass 1 (CG fit +
    predict) and its exchange, :299-307 the five smoothings, :311 the
    broadcast, :169-172 hyper lookup, :316-320 pass 2 and its gather -- the
    production output `_interp_smth` -- as day.interpolate_day on a binned
    synthetic 25 km day (synthetic.make_binned_day: ~1e4 ice cells, ~300-3000
    observations within 300 km).  A step is one whole day (seed + step)."""
    import tempfile
    from optimalinterpolation_amd import _lib, day as DAY, synthetic
    small = dict(nx=48, ice_radius_m=200e3, obs_radius_m=500e3, cover=(0.02, 0.06)) if args.twopass_small else {}
    days = [synthetic.make_binned_day(seed=args.seed + k, **small) for k in range(args.steps)]
    if not args.no_prime:
        w = synthetic.make_binned_day(seed=999, nx=40, ice_radius_m=110e3, obs_radius_m=450e3, cover=(0.02, 0.05))
        DAY.interpolate_day(w.sat, w.sie, w.x, w.y, w.mean, date='w', rank=rank, world=world, device=gpu,
                            comm_device=cdev)
    _lib.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = []
    for k, d in enumerate(days):
        res.append(DAY.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date=d.date, rank=rank, world=world,
                                       device=gpu, comm_device=cdev, profile=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank != 0:
        dist.destroy_process_group()
        return
    prof = _lib.profile_json()
    r0, d0 = res[0], days[0]
    ids = np.where(~np.isnan(d0.sie))
    ncell = int(sum(r.info['ncell'] for r in res))
    tim = {k: round(float(np.sum([r.info['timing'][k] for r in res])), 3)
           for k in ('neighbours_s', 'pass1_s', 'smooth_s', 'pass2_s', 'total_s')}
    evals = np.concatenate([np.asarray(r.info['evals'], float) for r in res])
    counts = np.concatenate([np.asarray(r.info['counts'], float) for r in res])
    # distinct sites per cell (the m x m problem the library solves), host-side for the flop model
    from scipy.spatial import cKDTree
    sites = []
    for d in days:
        xt, yt, tt_, _ = DAY.training_set(d.sat, d.x, d.y)
        idd = np.where(~np.isnan(d.sie))
        tree = cKDTree(np.column_stack([xt, yt]))
        key = np.column_stack([xt, yt, tt_]).view(np.dtype((np.void, 24))).ravel()
        for lst in tree.query_ball_point(np.column_stack([d.x[idd], d.y[idd]]), r=synthetic.RADIUS_M):
            sites.append(max(1, len(np.unique(key[np.asarray(lst, dtype=np.int64)]))))
    n = np.asarray(sites, float)
    ok = np.isfinite(evals)
    rl = roofline_of(prof, np.where(ok, evals, 0.0), n, dt, counts, extra_pred=1)
    line = {"metric": "grid-cells/sec (whole two-pass day: fit+predict, smooth, predict), 25 km, fp64",
            "value": round(ncell / dt, 4), "unit": "grid-cells/s", "n_gpus": world, "steps": args.steps,
            "warmup": 0, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic binned day (synthetic.make_binned_day: 320x320 grid, 4 satellites x 9 days)",
            "config": {"workload": ("the reference's whole day GPR_CS2S3.py:223-336 per step: training set, "
                                    "300 km query, pass 1 CG fit + predict, all-gather, 5 smoothings, hyper lookup, "
                                    "pass 2 predict (the production `_interp_smth`), gather; binned grids on the "
                                    "host, the training set assembled and uploaded inside the timed region"),
                       "day_cells": int(r0.info['ncell']), "n_train": int(r0.info['n_train']),
                       "obs_per_cell_mean": round(float(np.mean(counts)), 1),
                       "obs_per_cell_range": [int(counts.min()), int(counts.max())],
                       "parallelism": f"dp{world} (LPT cell partition; one all_gather after pass 1, one gather "
                                      f"after pass 2)"},
            "stages_s": tim, "pass2_share": round(tim['pass2_s'] / max(tim['total_s'], 1e-12), 5),
            "pass2_cells_per_s": round(ncell / max(tim['pass2_s'], 1e-12), 1),
            "evals_per_cell": round(float(np.mean(evals[ok])), 2), "failed_cells": int(np.sum(~ok)),
            "roofline": rl, **args.dist_fields}
    # parity: smoothing bit-exact on the GPU's own pass-1 fields; pass 2 of sampled cells at T1
    tmp = tempfile.mkdtemp(prefix='oi_twopass_')
    path = os.path.join(tmp, 'day.npz')
    p1 = np.stack([r0[d0.date + '_' + k] for k in DAY.HYPER_KEYS])
    sm = np.stack([r0[d0.date + '_' + k + '_smth'] for k in DAY.HYPER_KEYS])
    order = np.argsort(counts[:len(ids[0])], kind='stable')
    pick = np.array([int(b[len(b) // 2]) for b in np.array_split(order, max(1, args.parity_cells)) if len(b)])
    np.savez(path, sat=d0.sat, sie=d0.sie, x=d0.x, y=d0.y, mean=d0.mean, T=synthetic.T_DAYS, radius=300.0,
             std=DAY.smooth_std(25), p1=p1, sm=sm, cells=pick,
             hyp=np.column_stack([s_[ids][pick] for s_ in sm]),
             fs=r0[d0.date + '_interp_smth'][ids][pick], sd=r0[d0.date + '_interp_error_smth'][ids][pick])
    deadline = time.time() + 600
    chk = run_argv_jobs(TWOPASS_CHECK, [[path, 'smooth']] +
                        [[path, 'pass2']], 2, deadline)
    par = {"cells": int(len(pick)), "tol": 1e-10}
    if chk[0] is not None:
        par["smooth_bit_exact"] = chk[0]["smooth_bit_exact"]
    if chk[1] is not None:
        par.update(max_rel_fs=chk[1]["max_rel_fs"], max_rel_sd=chk[1]["max_rel_sd"],
                   n_min=min(chk[1]["n"]), n_max=max(chk[1]["n"]))
    par["pass"] = bool(chk[0] is not None and chk[1] is not None and all(par["smooth_bit_exact"])
                       and par["max_rel_fs"] <= 1e-10 and par["max_rel_sd"] <= 1e-10)
    par["note"] = ("day 0: the oracle's smoothing (GPR:65-76 restated) of the GPU's pass-1 fields vs the GPU's "
                   "smoothed fields (bitwise), and the oracle's GPR3D(opt=False) with the reference's cKDTree "
                   "neighbour order at the GPU's smoothed hypers vs the GPU's pass-2 fs / sd on a stratified "
                   "sample of cells (T1)")
    line["parity"] = par
    if world == 1 and not args.no_cpu_baseline:
        workers, desc = host_cores(args)
        try:
            line["cpu_baseline"] = cpu_baseline(counts[ok], evals[ok], workers, desc, time.time() + 400,
                                                extra_pred=1)
        except Exception as e:
            line["cpu_baseline"] = {"value": None, "error": repr(e)}
    else:
        line["cpu_baseline"] = None
    s = json.dumps(line)
    print(s, flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            f.write(s + '\n')
    if world > 1:
        dist.destroy_process_group()


# ----------------------------------------------------------------- launcher
def visible_gpus():
    """GPUs a rank process will see, counted in a child process: the launcher
    itself never initialises HIP (a process that has must not start the
    ranks)."""
    out = subprocess.run([sys.executable, '-c', 'import torch; print(torch.cuda.device_count())'],
                         capture_output=True, text=True, timeout=600)
    lines = out.stdout.strip().splitlines()
    if out.returncode != 0 or not lines:
        raise RuntimeError(f"GPU count probe failed (rc {out.returncode}): {out.stderr[-400:]}")
    return int(lines[-1])


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def launch_ranks(n, argv, script=None, gpus=None, backend=None, grace_s=20.0, poll_s=0.25, deadline_s=None):
    """`bench.py --gpus N` without a launcher around it: start N rank
    processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT in their environment, the torch.distributed.run contract),
    forward rank 0's stdout (the JSON line) and every rank's stderr, and return
    the exit code: 0 only if every rank exited 0 and rank 0 printed a JSON
    line.  The first rank to fail ends the others (SIGTERM, then SIGKILL after
    ``grace_s``) and its code is returned.  Called before this process imports
    anything that touches the GPU; ranks are started as children, never by
    exec.  ``gpus``: visible GPU count (probed in a child when None); N > gpus
    is refused (exit 2) unless the backend is gloo.  ``deadline_s`` (seconds
    from T_PROC): ranks still running then -- e.g. one stuck in a
    collective after another exited 0 -- are ended and 124 is returned."""
    import signal
    import threading
    backend = backend or os.environ.get('OI_DIST_BACKEND', 'nccl')
    script = script or os.path.abspath(__file__)
    if gpus is None:
        gpus = visible_gpus()
    if n > gpus and backend != 'gloo':
        log(f"--gpus {n} but only {gpus} GPU(s) visible: refusing to oversubscribe "
            f"(OI_DIST_BACKEND=gloo rehearses N ranks on one GPU)")
        return 2
    port = free_port()
    procs, lines = [], []

    def pump(stream):  # rank 0's stdout -> ours, remembering the JSON lines
        for ln in stream:
            sys.stdout.write(ln)
            sys.stdout.flush()
            if ln.lstrip().startswith('{'):
                lines.append(ln.strip())
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                   OI_BENCH_LAUNCHER='bench.py', OI_BENCH_T0=repr(T_PROC))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env, text=True,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    th = threading.Thread(target=pump, args=(procs[0].stdout,), daemon=True)
    th.start()

    def end_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)
        t_end = time.time() + grace_s
        for p in procs:
            while p.poll() is None and time.time() < t_end:
                time.sleep(0.05)
            if p.poll() is None:
                p.kill()
                p.wait()
    prev = signal.signal(signal.SIGTERM, lambda *_: (end_all(), sys.exit(143)))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                log(f"rank {procs.index(bad[0])} exited with {rc}: ending the other ranks")
                end_all()
                break
            if deadline_s is not None and elapsed() > deadline_s:
                live = [r for r, p in enumerate(procs) if p.poll() is None]
                log(f"launcher deadline {deadline_s:.0f} s passed with ranks {live} still running: ending them")
                end_all()
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        signal.signal(signal.SIGTERM, prev)
    th.join(timeout=5.0)
    if rc == 0:
        codes = [p.returncode for p in procs]
        rc = next((c for c in codes if c != 0), 0)
        if rc == 0 and not lines:
            log("rank 0 printed no JSON line")
            rc = 1
    return rc if rc > 0 else (128 - rc if rc < 0 else 0)


def rank_census(dist, torch, world, rank, gpu, cdev):
    """[(rank, device index)] of every rank, by one all_gather: the line
    reports which ranks took part and on which GPUs (``ranks_seen``)."""
    if world == 1:
        return [(0, gpu)]
    mine = torch.tensor([rank, gpu], dtype=torch.int64, device=cdev)
    allr = [torch.zeros(2, dtype=torch.int64, device=cdev) for _ in range(world)]
    dist.all_gather(allr, mine)
    return sorted((int(t[0].item()), int(t[1].item())) for t in allr)


def dist_fields(census, backend, world, args):
    ndev = len({g for _, g in census})
    return {"ranks_seen": [r for r, _ in census], "rank_devices": [g for _, g in census],
            "collective_backend": (backend if world > 1 else None), "gpus_requested": args.gpus,
            "distinct_devices": ndev,
            "launcher": os.environ.get('OI_BENCH_LAUNCHER',
                                       'torch.distributed.run' if 'TORCHELASTIC_RUN_ID' in os.environ
                                       else ('external' if world > 1 else 'none'))}


# ----------------------------------------------------------------- main
def heartbeat(period=60.0):
    """One stderr line a minute (batch runners take a long silence for a hang)."""
    import threading

    def beat():
        while True:
            time.sleep(period)
            print(f"[bench {elapsed():6.1f}s] running", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def per_rank_record(rank, cells, dt, outs, done_k, opt, tprof):
    """[rank, cells fitted, own timed seconds, SMLII evaluations, GPU ms of the
    rounds with < 256 resident cells (-1 without per-launch profiling)]."""
    from optimalinterpolation_amd import _lib
    ev = float(sum(float(np.sum(outs[k][2][:, 3])) for k in range(done_k))) if opt else 0.0
    tail = -1.0
    if tprof:
        rl = _lib.profile_json().get('rounds_log') or []
        tail = float(sum(r[4] for r in rl if r[0] + r[1] < 256))
    return [rank, float(cells), float(dt), ev, tail]


def site_counts(cells):
    """Distinct (x, y, t) sites per cell: the size of the problem the library
    solves (oi_device.h "Duplicate sites"); host-side, for the flop model."""
    v = np.ascontiguousarray(cells.xyt).view(np.dtype((np.void, 24))).ravel()
    return np.array([len(np.unique(v[a:b])) for a, b in zip(cells.offs[:-1], cells.offs[1:])], dtype=np.int64)


def roofline_of(prof, evals, n, dt, n_obs=None, extra_pred=0):
    """Roofline of the dominant kernel from the library's HIP-event profile
    (every launch of the timed region, on the stream the kernels run on).
    ``n``: the solved size per cell (distinct sites); ``n_obs``: observations
    (the reference's n x n problem) for the reference-equivalent rate."""
    kern = prof['kernels']
    gemm = {k: v for k, v in kern.items() if v['flops'] > 0 and v['total_ms'] > 0}
    dom = max(gemm, key=lambda k: gemm[k]['total_ms']) if gemm else max(kern, key=lambda k: kern[k]['total_ms'])
    kd = kern[dom]
    achieved_exec = kd['flops'] / (kd['total_ms'] / 1e3) / 1e12 if kd['total_ms'] > 0 else 0.0
    # algorithmic flops of the dominant kernel (SURVEY §8d per-unit figures):
    # the factor family (k_panel4, k_panel_even, k_chol_panel) carries potrf +
    # trtri = 2n^3/3 per evaluation and potrf n^3/3 per predict, k_lauum_grad
    # the lauum n^3/3 per evaluation; each kernel gets its family's algorithmic
    # flops in proportion to its share of the family's executed tile products.
    fam_alg = {'factor': float(np.sum((evals * 2.0 / 3.0 + (1.0 + extra_pred) / 3.0) * n ** 3)),
               'lauum': float(np.sum(evals * n ** 3 / 3.0))}
    fam_of = {'k_panel_even': 'factor', 'k_panel4': 'factor', 'k_chol_panel': 'factor',
              'k_lauum_grad': 'lauum'}
    fam = fam_of.get(dom)
    fam_exec = sum(v['flops'] for k, v in kern.items() if fam_of.get(k) == fam) if fam else 0.0
    alg_dom = kd['flops'] * fam_alg[fam] / fam_exec if fam and fam_exec > 0 else kd['flops']
    achieved = alg_dom / (kd['total_ms'] / 1e3) / 1e12 if kd['total_ms'] > 0 else 0.0
    # every GEMM kernel on the same footing (algorithmic and executed rates),
    # and each family's executed / algorithmic flops (padding + O(T^2) products)
    per_kernel = {}
    for k, v in kern.items():
        f = fam_of.get(k)
        if not f or v['total_ms'] <= 0:
            continue
        fe = sum(x['flops'] for kk, x in kern.items() if fam_of.get(kk) == f)
        alg = v['flops'] * fam_alg[f] / fe if fe > 0 else 0.0
        per_kernel[k] = {"alg_tflops": round(alg / (v['total_ms'] / 1e3) / 1e12, 3),
                         "frac": round(alg / (v['total_ms'] / 1e3) / 1e12 / PEAK_FP64_TFLOPS, 4),
                         "exec_tflops": round(v['flops'] / (v['total_ms'] / 1e3) / 1e12, 3),
                         "ms": round(v['total_ms'], 3)}
    fam_ratio = {}
    for f in ('factor', 'lauum'):
        fe = sum(x['flops'] for kk, x in kern.items() if fam_of.get(kk) == f)
        if fam_alg[f] > 0 and fe > 0:
            fam_ratio[f] = round(fe / fam_alg[f], 4)
    traffic = None
    tfile = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(tfile):
        try:
            traffic = json.load(open(tfile)).get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    npred = 1 + extra_pred  # predict blocks per cell (pass 2 of the two-pass day adds one)
    useful = float(np.sum(evals * (n ** 3 + 40 * n ** 2) + npred * (n ** 3 / 3 + 16 * n ** 2)))
    no = n if n_obs is None else n_obs
    ref_eq = float(np.sum(evals * (no ** 3 + 40 * no ** 2) + npred * (no ** 3 / 3 + 16 * no ** 2)))
    return {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": PEAK_FP64_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP64_TFLOPS, 4), "traffic": traffic,
            "traffic_note": ("HBM bytes per launch of this kernel, rocprofv3 PMC FETCH_SIZE(x2, gfx950)+WRITE_SIZE, "
                             "profiles/pmc_traffic.json") if traffic is not None else None,
            "launches": kd['launches'], "avg_launch_ms": kd['total_ms'] / max(kd['launches'], 1),
            "flops_per_launch": alg_dom / max(kd['launches'], 1),
            "flop_model": ("algorithmic: SURVEY §8d potrf+trtri 2m^3/3 per eval (+ potrf m^3/3 per predict) "
                           "for the factor kernels, lauum m^3/3 per eval for k_lauum_grad, m = the cell's "
                           "distinct sites (the m x m problem solved, oi_device.h), unpadded, split over a "
                           "family's kernels by executed tile products"),
            "achieved_executed": round(achieved_exec, 3),
            "frac_executed": round(achieved_exec / PEAK_FP64_TFLOPS, 4),
            "executed_flops_per_launch": kd['flops'] / max(kd['launches'], 1),
            "executed_flop_model": ("executed fp64 MFMA flops: the 16x16 blocks x 16-deep chunks the kernels issue "
                                    "(padding, triangular-operand and zero chunks they skip are not counted; the "
                                    "engine mirrors the kernels' masks, oi_masks.h)"),
            "kernels_ms": {k: round(v['total_ms'], 3) for k, v in kern.items() if v['launches']},
            "gemm_kernels": per_kernel,
            "executed_over_algorithmic": fam_ratio,
            "useful_tflops_per_gpu": round(useful / dt / 1e12, 3),
            "useful_frac_per_gpu": round(useful / dt / 1e12 / PEAK_FP64_TFLOPS, 4),
            "useful_flop_model": "SURVEY §8d: E*(m^3+40m^2) + m^3/3 + 16m^2 per cell, m distinct sites",
            "reference_equivalent_tflops_per_gpu": round(ref_eq / dt / 1e12, 3),
            "reference_equivalent_model": ("the same formula on n observations: the n x n work the reference's "
                                           "algorithm does per cell, / the measured time"),
            "sites_over_obs_mean": round(float(np.mean(n / np.maximum(no, 1))), 4)}


def main():
    args = parse()
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        # no launcher around us: start the ranks ourselves, before any GPU call
        # deadline: the slice budget + the rank-0 parity check / teardown
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], deadline_s=args.budget_s + LAUNCH_GRACE_S))
    heartbeat()
    # one resident-cell group (one stream): OI_GROUPS=2 overlaps one group's
    # latency-bound launches with the other's GEMMs, +0.5 % on the day
    # (profiles/r02/ab/), but the two streams' kernels then share the chip and
    # the per-kernel HIP-event durations the roofline divides by stop being
    # the kernel's own (frac 0.46 vs 0.61 on the same run)
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # collectives: RCCL ('nccl') by default; OI_DIST_BACKEND=gloo (collective
    # payloads staged on the host) lets several ranks share one GPU, which is
    # how the N>1 path is rehearsed on a 1-GPU box
    backend = os.environ.get('OI_DIST_BACKEND', 'nccl')
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}: the line would "
                         f"misreport n_gpus")
    ndev = torch.cuda.device_count()
    if local >= ndev and backend != 'gloo':
        raise SystemExit(f"bench.py: LOCAL_RANK {local} but {ndev} GPU(s) visible: refusing to put two "
                         f"ranks on one GPU (OI_DIST_BACKEND=gloo for a one-GPU rehearsal)")
    gpu = local % max(1, ndev)
    # ranks sharing one GPU (the gloo rehearsal): this node's ranks, not the
    # global world (2 nodes x 8 GPUs must not halve every arena)
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', '') or world)
    per_dev = -(-local_world // max(1, ndev))
    if per_dev > 1:  # each rank's library arena takes a share of the HBM, not 60 % of what is left
        os.environ.setdefault('OI_ARENA_FRAC', f"{0.8 / per_dev:.4f}")
    # the rank's device is current before the process group exists, so RCCL's
    # communicator binds to this GPU and not to the rank-guessed default
    torch.cuda.set_device(gpu)
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group(backend)
    dev = torch.device('cuda', gpu)
    cdev = torch.device('cpu') if backend == 'gloo' else dev  # where collective tensors live
    census = rank_census(dist, torch, world, rank, gpu, cdev)
    args.dist_fields = dist_fields(census, backend, world, args)
    if rank == 0:
        log(f"world {world}: ranks {args.dist_fields['ranks_seen']} on devices "
            f"{args.dist_fields['rank_devices']} ({backend if world > 1 else 'no collectives'})")
    if args.workload == 'nystrom':
        if args.depth is None:
            args.depth = 8
        return main_nystrom(args, torch, dist, world, rank, gpu, cdev)
    if args.workload == 'svgp':
        return main_svgp(args, torch, dist, world, rank, gpu, cdev)
    if args.workload == 'twopass':
        return main_twopass(args, torch, dist, world, rank, gpu, cdev)
    from optimalinterpolation_amd import _lib, synthetic

    slices, warm, opt, cfg, scaling, counts_all = build_slices(args, rank, world)
    if args.depth is None:
        args.depth, cfg["depth_rule"] = default_depth(args, world, len(slices), cfg.get("slices_per_day"))
    cfg["depth"] = args.depth
    x0 = X0_12P5 if args.workload == 'season' else X0
    log(f"rank {rank}: {len(slices)} slices, {sum(s.ncell for s in slices)} cells")

    def resident(cells):  # inputs in HBM before timing
        h = None if opt else np.tile(synthetic.FIXED_HYPERS, (cells.ncell, 1))
        return (cells, torch.from_numpy(cells.xyt).to(dev).contiguous(),
                torch.from_numpy(cells.z).to(dev).contiguous(), h)
    dev_slices = [resident(c) for c in slices]
    dev_warm = [resident(c) for c in warm]
    torch.cuda.synchronize()

    def submit(sess, item):
        cells, xyt, z, h = item
        return sess.submit(xyt, z, cells.offs, cells.xs, cells.mean, x0=x0 if opt else None, opt=opt, hyp=h)

    # day / season: the neighbour query and gather (GPR:159-161) inside the
    # timed region, over the rank's cells pooled into one training set
    pool = None
    if args.workload in ('day', 'days', 'season') and not args.pregathered:
        pool = pool_training_set(slices, synthetic.GRID_12P5_M if args.workload == 'season' else synthetic.GRID_M,
                                 torch, dev)
        cfg["neighbour_query"] = (f"inside the timed region: per slice oi_ball_query (r = {pool['r'] / 1e3:.0f} km) "
                                  f"over the rank's {pool['M']} observations pooled into one HBM-resident training "
                                  f"set, then oi_gather_rows (GPR:159-161); the searched positions are cell g's "
                                  f"observations translated to node g of a {POOL_PITCH_M / 1e3:.0f} km lattice, "
                                  f"the gathered columns the observations as drawn")

    def submit_queried(sess, k):
        cells = slices[k]
        offs, idx = _lib.ball_query_device(pool['pts'], pool['q'][k], pool['r'])
        if not np.array_equal(offs, cells.offs):
            raise RuntimeError(f"slice {k}: the radius query returned other observations than the cells' own")
        xyt, z = _lib.gather_rows_device(pool['cols'], idx)
        return sess.submit(xyt, z, cells.offs, cells.xs, cells.mean, x0=x0, opt=True)

    # library initialisation (context, arena, code objects): one untimed
    # one-shot call on 8 small cells -- not a step
    if not args.no_prime:
        prime = synthetic.make_cells([300] * 8, seed=12345)
        _lib.gpr_batch(prime.xyt, prime.z, prime.offs, prime.xs, prime.mean, x0=X0, opt=True, device=gpu,
                       profile=True)
    single = args.workload == 'single'
    # (season too: its profiled second pass would repeat the whole timed run)
    tprof = (args.workload in ('day', 'days', 'season')) if args.timed_profile == 'auto' else args.timed_profile == 'on'
    sess = None if single else _lib.Session(device=gpu, device_inputs=True, profile=tprof, max_pool=args.max_pool)
    if single:  # config 1: blocking one-shot calls (per-cell latency)
        for item in dev_warm:
            cells, xyt, z, h = item
            _lib.gpr_batch_device(xyt, z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True, device=gpu)
    else:
        for item in dev_warm:
            submit(sess, item)
        sess.wait(-1)
        if pool is not None:  # the query / gather code paths, untimed
            _lib.gather_rows_device(pool['cols'], _lib.ball_query_device(pool['pts'], pool['q'][0], pool['r'])[1])
    prof_untimed = _lib.profile_json()['kernels']  # priming + warmup launches (rocprof sees them too)
    _lib.profile_reset()
    log("warmup done; timing")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs, tickets, done_k, truncated = {}, [], 0, False
    for k, item in enumerate(dev_slices):
        if elapsed() > args.budget_s:
            truncated = True
            log(f"budget {args.budget_s:.0f} s reached: {k} of {len(dev_slices)} slices submitted")
            break
        if single:  # per-launch events would add ~40 % to a one-cell call: timed unprofiled
            cells, xyt, z, h = item
            outs[k] = _lib.gpr_batch_device(xyt, z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True,
                                            info=True, device=gpu, profile=False)
        else:
            tickets.append(submit_queried(sess, k) if pool is not None else submit(sess, item))
            if k >= args.depth:
                outs[k - args.depth] = sess.wait(tickets[k - args.depth])
        done_k = k + 1
    for k in range(done_k):
        if k not in outs:
            outs[k] = sess.wait(tickets[k])
    t_own = time.perf_counter() - t0  # this rank's own work done (before the gather and the closing barrier)
    # the single gather of posterior fields (ncell x 8 fp64) to rank 0
    rows = np.concatenate([outs[k][0] for k in range(done_k)]) if done_k else np.zeros((0, 8))
    if world > 1:
        # every rank takes the same collective path: the row counts are always
        # exchanged (one tiny all_gather), since a rank that hit --budget-s on
        # its own clock holds fewer rows than the partition gave it
        cs = [torch.zeros(1, dtype=torch.int64, device=cdev) for _ in range(world)]
        dist.all_gather(cs, torch.tensor([rows.shape[0]], dtype=torch.int64, device=cdev))
        kmax = int(max(int(c.item()) for c in cs))
        pay = torch.zeros((max(kmax, 1), 8), dtype=torch.float64, device=cdev)
        pay[:rows.shape[0]] = torch.from_numpy(rows).to(cdev)
        bufs = [torch.empty_like(pay) for _ in range(world)] if rank == 0 else None
        dist.gather(pay, bufs, dst=0)
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if sess is not None:
        sess.close()
    ncells_rank = sum(slices[k].ncell for k in range(done_k))
    # per-rank evidence (GPR:256,262's scatter/gather): every
    # rank's cells, the seconds until its own last slice was done (the timed
    # region itself ends at a common barrier), SMLII evaluations and the GPU
    # time of its tail rounds (< 256 resident cells), so the scaling line shows
    # imbalance
    per_rank = [per_rank_record(rank, ncells_rank, t_own, outs, done_k, opt, tprof)]
    if world > 1:
        mine = torch.tensor(per_rank[0][1:], dtype=torch.float64, device=cdev)
        allr = [torch.zeros(4, dtype=torch.float64, device=cdev) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [[r] + [float(v) for v in t.tolist()] for r, t in enumerate(allr)]
        tt = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    tot = torch.tensor([float(ncells_rank)], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(tot)
    total_cells = float(tot.item())
    log(f"GPU leg: {total_cells:.0f} cells in {dt:.2f} s = {total_cells / dt:.3f} cells/s")

    if single:  # the roofline's per-launch times: the same calls again, profiled, untimed
        _lib.profile_reset()
        for k in range(done_k):
            cells, xyt, z, h = dev_slices[k]
            _lib.gpr_batch_device(xyt, z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True, device=gpu,
                                  profile=True)
    elif not tprof:  # the same slices again through a profiled session, untimed
        _lib.profile_reset()
        psess = _lib.Session(device=gpu, device_inputs=True, profile=True, max_pool=args.max_pool)
        for k in range(done_k):
            submit(psess, dev_slices[k])
        psess.wait(-1)
        psess.close()
    prof = _lib.profile_json()
    info = np.concatenate([outs[k][2] for k in range(done_k)])
    status = np.concatenate([outs[k][1] for k in range(done_k)])
    sizes_timed = np.concatenate([np.diff(slices[k].offs) for k in range(done_k)])
    sites_timed = np.concatenate([site_counts(slices[k]) for k in range(done_k)])
    evals = info[:, 3].astype(float) if opt else np.zeros(len(sizes_timed))
    n = sites_timed.astype(float)
    metric = (METRIC if args.workload in ('day', 'days') else
              "grid-cells/sec (full GP fit+predict), 12.5 km season, fp64" if args.workload == 'season' else
              f"grid-cells/sec ({args.workload}), fp64")
    line = {"metric": metric,
            "value": round(total_cells / dt, 4), "unit": "grid-cells/s", "n_gpus": world,
            "steps": done_k, "warmup": args.warmup, "ms_per_step": round(dt / max(done_k, 1) * 1e3, 3),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded SURVEY §8d generator; reference data not shipped)",
            "config": cfg, "evals_per_cell": round(float(np.mean(evals)), 2) if opt else 0,
            "failed_cells": int(np.sum(status != 0)), "timed_s": round(dt, 3),
            "roofline": roofline_of(prof, evals, n, dt, sizes_timed.astype(float)), **args.dist_fields}
    line["per_rank"] = [{"rank": int(r), "cells": int(c), "own_work_s": round(t, 3), "evals": int(e),
                         "tail_round_gpu_ms": (round(m, 1) if m >= 0 else None)} for r, c, t, e, m in per_rank]
    if world > 1:
        line["config"]["cells_per_rank"] = [int(c) for c in counts_all]
    if not tprof:
        line["roofline"]["timing_note"] = ("per-launch HIP-event times from a second, profiled pass over the "
                                           "same cells; the timed pass runs without per-launch events")
    rl = prof.get('rounds_log') or []
    if rl:  # [n_eval, n_pred, maxT, sum T^3 of fitting cells, GPU ms] per round
        tot = sum(r[4] for r in rl)
        small = [r for r in rl if r[0] + r[1] < 256]
        line["host"] = {k: round(prof.get(k, 0.0), 3) for k in ('wall_s', 'sync_s', 'consume_s', 'prep_s', 'launch_s')}
        line["rounds"] = {"count": len(rl), "gpu_ms": round(tot, 1),
                          "lt256_cells": len(small), "lt256_gpu_ms": round(sum(r[4] for r in small), 1),
                          "note": "rounds with < 256 resident cells (the day's tail of slow-converging cells)"}
    dom = line["roofline"]["kernel"]
    pu, pt = prof_untimed.get(dom, {"launches": 0, "total_ms": 0.0}), prof["kernels"][dom]
    nall = pu["launches"] + pt["launches"]
    line["roofline"]["rocprof_crosscheck"] = {
        "launches_incl_untimed": nall,
        "avg_launch_ms_incl_untimed": (pu["total_ms"] + pt["total_ms"]) / max(nall, 1),
        "note": "HIP-event average over every launch of the process (priming + warmup + timed), the set a "
                "rocprofv3 --kernel-trace --stats run of this command averages over"}
    if done_k != args.steps or truncated:
        line.update({"truncated": True, "steps_requested": args.steps})
    if args.dump and rank == 0:  # per (kernel, block column) launch totals of the profiled pass
        with open(args.dump + '.byj.json', 'w') as fh:
            json.dump(prof.get('by_j', []), fh)
    if args.dump:
        np.savez(args.dump if rank == 0 else f"{args.dump}.rank{rank}.npz", n=sizes_timed, m=sites_timed,
                 evals=info[:, 3], nit=info[:, 0], cg_status=info[:, 1], status=status)
    if rank == 0:
        log("line (before cpu_baseline): " + json.dumps({k: line[k] for k in ('value', 'steps', 'ms_per_step')}))
    if rank == 0 and opt and args.parity_cells > 0 and args.workload in ('day', 'days', 'season'):
        try:
            timed = [slices[k] for k in range(done_k)]
            rows = np.concatenate([outs[k][0] for k in range(done_k)])
            line["parity"] = timed_parity(timed, rows, status, args.parity_cells, gpu,
                                          T_PROC + args.budget_s + 10.0, host_cores(args)[0])
        except Exception as e:  # never lose the GPU line over the check
            line["parity"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and opt and args.workload != 'single':
        workers, desc = host_cores(args)
        if args.workload == 'season':
            global EVAL_PROBES
            EVAL_PROBES = (300, 1000, 2000, 3000, 4000, 5000)
        deadline = T_PROC + args.budget_s + 20.0
        if time.time() + 30 > deadline:
            line["cpu_baseline"] = {"value": None, "error": "skipped: wall-clock budget spent by the GPU leg"}
        else:
            try:
                line["cpu_baseline"] = cpu_baseline(sizes_timed, evals, workers, desc, deadline)
            except Exception as e:  # never lose the GPU line over the baseline
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and not opt:
        workers, desc = host_cores(args)
        line["cpu_baseline"] = cpu_predict_baseline(workers, desc)
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and single:
        workers, desc = host_cores(args)
        line["cpu_baseline"] = cpu_single_baseline([args.seed + 31 * k for k in range(done_k)], workers, desc)
    else:
        line["cpu_baseline"] = None
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, 'w') as f:
                f.write(s + '\n')
    if world > 1:
        dist.destroy_process_group()


CHECK_JOB = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import gp_oracle as O
d = np.load(sys.argv[2])
x, y, xs, mean, hyp = d['x'], d['y'], d['xs'], float(d['mean']), d['hyp']
h = np.r_[np.log(hyp), np.log(.1)]
f, g = O.neg_log_ml(h, x, y, np.ones(len(y)) * mean)
fs, sd, lz = O.predict(x, y, xs, mean, hyp[:3], hyp[3], hyp[4])
# S_j = 1/2 sum |Q o dK_j|: the magnitude of what the gradient sums (tests/test_gpu_parity.py)
n = len(y)
K, dK = O.matern32(x, hyp[:3], hyp[3], grad=True)
Kinv = np.linalg.inv(K + np.eye(n) * hyp[4])
a = Kinv @ (y - mean)
Q = Kinv - np.outer(a, a)
S = [np.abs(Q * dK[j]).sum() / 2 for j in range(3)] + [np.abs(Q * 2 * K).sum() / 2,
                                                      hyp[4] * np.abs(np.diag(Q)).sum(), 0.0]
print(json.dumps({"nlz": float(np.asarray(f).ravel()[0]), "grad": [float(v) for v in np.ravel(g)],
                  "gscale": [float(v) for v in S],
                  "fs": float(np.ravel(fs)[0]), "sd": float(np.ravel(sd)[0]), "lz": float(np.ravel(lz)[0])}))
'''


def timed_parity(timed, rows, status, k, gpu, deadline, workers):
    """T1 parity of the bench's own timed cells: a stratified
    sample of ``k`` timed cells (equal-count n buckets, spread inside each),
    the GPU's objective (oi_nlml_grad_batch, SMLII GPR:107-141) and the fitted
    cells' posterior (fs, sd, lZ: the timed run's own output rows, GPR:173-182)
    against the CPU oracle (bit-exact restatement of GPR:78-191) at the hypers
    the GPU fit found.  Tolerance 1e-10 relative (max(1, |ref|)); the gradient
    as |dg| <= 1e-10 (|g| + S_j), S_j = 1/2 sum |Q o dK_j| (tests/test_gpu_parity.py)."""
    import tempfile
    from optimalinterpolation_amd import _lib, synthetic
    cells = [(t, c) for t in timed for c in range(t.ncell)]
    sizes = np.array([t.offs[c + 1] - t.offs[c] for t, c in cells])
    ok = np.flatnonzero(status == 0)
    order = ok[np.argsort(sizes[ok], kind='stable')]
    pick = [int(b[len(b) // 2]) for b in np.array_split(order, min(k, len(order))) if len(b)]
    sub = synthetic.RaggedCells(np.concatenate([cells[p][0].cell(cells[p][1])[0] for p in pick]),
                                np.concatenate([cells[p][0].cell(cells[p][1])[1] for p in pick]),
                                np.concatenate([[0], np.cumsum(sizes[pick])]),
                                np.concatenate([cells[p][0].cell(cells[p][1])[2] for p in pick]),
                                timed[0].mean)
    hyp = rows[pick, 3:8]
    h6 = np.column_stack([np.log(hyp), np.full(len(pick), np.log(.1))])
    nlz, grad, st = _lib.nlml_grad_batch(sub.xyt, sub.z, np.full(len(sub.z), sub.mean), sub.offs, h6, device=gpu)
    tmp = tempfile.mkdtemp(prefix='oi_parity_')
    jobs = []
    for q in range(len(pick)):
        x, y, xs = sub.cell(q)
        path = os.path.join(tmp, f'c{q}.npz')
        np.savez(path, x=x, y=y, xs=xs, mean=sub.mean, hyp=hyp[q])
        jobs.append([path])
    res = run_argv_jobs(CHECK_JOB, jobs, workers, deadline)
    rel = lambda a, b: abs(a - b) / max(1.0, abs(b))
    worst = {"nlz": 0.0, "grad": 0.0, "fs": 0.0, "sd": 0.0, "lz": 0.0}
    checked = 0
    for q, r in enumerate(res):
        if r is None:
            continue
        checked += 1
        worst["nlz"] = max(worst["nlz"], rel(nlz[q], r["nlz"]))
        g = np.array(r["grad"])
        sc = np.maximum(np.abs(g) + np.array(r["gscale"]), 1e-300)
        worst["grad"] = max(worst["grad"], float(np.max(np.abs(grad[q] - g) / sc)))
        for key, col in (("fs", 0), ("sd", 1), ("lz", 2)):
            worst[key] = max(worst[key], rel(rows[pick[q], col], r[key]))
    n_chk = [int(sizes[pick[q]]) for q in range(len(pick)) if res[q] is not None]
    return {"cells": checked, "n_min": min(n_chk) if n_chk else None, "n_max": max(n_chk) if n_chk else None,
            "max_rel_nlz": worst["nlz"], "max_rel_grad": worst["grad"], "max_rel_fs": worst["fs"],
            "max_rel_sd": worst["sd"], "max_rel_lz": worst["lz"], "tol": 1e-10,
            "pass": bool(checked == len(pick) and max(worst.values()) <= 1e-10 and np.all(st == 0)),
            "note": ("T1 at the GPU fit's hypers: the timed run's fs/sd/lZ rows and oi_nlml_grad_batch's nlZ/"
                     "gradient vs oracle/gp_oracle.py (n x n, duplicate sites included) on a stratified sample "
                     "of the timed cells, CPU processes on the host after the timed region")}


def run_argv_jobs(script, jobs, workers, deadline):
    """``script`` in single-threaded-BLAS subprocesses, one per argument list in
    ``jobs`` (``workers`` at a time); -> parsed JSON per job (None if it failed
    or was not started before ``deadline``)."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    res = [None] * len(jobs)
    pending, running = list(range(len(jobs))), []
    while pending or running:
        while pending and len(running) < workers and time.time() < deadline:
            q = pending.pop(0)
            running.append((q, subprocess.Popen([sys.executable, '-c', script, ROOT] + [str(a) for a in jobs[q]],
                                                stdout=subprocess.PIPE, text=True, env=env)))
        if pending and time.time() >= deadline:
            pending = []
        for q, p in list(running):
            if p.poll() is not None:
                out = p.stdout.read()
                running.remove((q, p))
                if p.returncode == 0 and out.strip():
                    res[q] = json.loads(out.strip().splitlines()[-1])
        time.sleep(0.05)
    return res


def cpu_single_baseline(seeds, workers, desc):
    """Config 1 on the CPU: the oracle's full GPR3D(opt=True) (GPR:143-191 with
    scipy's CG) on the same n = 200 cells the GPU leg timed, each fit in its
    own single-threaded-BLAS process (one cell per MPI rank in the reference);
    the latency metric is one cell at a time, so value = 1 / mean fit time on
    one core (the fits run ``workers`` at a time only to finish sooner)."""
    res = run_jobs([('fit', 200, sd) for sd in seeds], workers, time.time() + 120)
    if not res:
        return {"value": None, "error": "no CPU fit finished"}
    t = float(np.mean([r['fit_s'] for r in res]))
    return {"value": 1.0 / t, "unit": "grid-cells/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/gp_oracle.py GPR3D(opt=True) on the {len(res)} timed n=200 cells, one "
                       f"single-threaded-BLAS process per cell, mean fit {t * 1e3:.1f} ms, "
                       f"{float(np.mean([r['evals'] for r in res])):.1f} evaluations/cell ({desc})")}


def cpu_predict_baseline(workers, desc):
    """Config 2 on the CPU: the oracle's predict block (GPR:173-182) at n = 500,
    timed while ``workers`` single-threaded-BLAS processes run at once."""
    jobs = [('eval', 500, 17 + r) for r in range(max(workers, 3))]
    res = run_jobs(jobs, workers, time.time() + 120)
    tp = float(np.median([r['pred_s'] for r in res]))
    return {"value": workers / tp, "unit": "grid-cells/s", "cores": workers, "kind": "port",
            "sample": (f"oracle/gp_oracle.py predict (GPR:173-182) at n=500, median of {len(res)} timings "
                       f"with {workers} processes at once ({desc})")}


if __name__ == '__main__':
    main()
