"""GPU parity of the day-level device steps against
the CPU restatements in oracle/day_oracle.py, through the C ABI.

  smoothing (GPR:65-76)        bit-exact vs the restatement (same window order,
                               no FMA, numpy's nanmean summation order)
  ball query (GPR:159)         exact index sets == scipy cKDTree (sorted)
  gather (GPR:160-161)         bit-exact
  day pipeline (GPR:200-336)   smoothed hyper fields bit-exact; pass-2 fields
                               (interp_smth, interp_error_smth) within
                               1e-10 * max(1, |ref|) (T1) of the oracle's
                               GPR3D(opt=False) on the same smoothed hypers
"""
import numpy as np
import pytest
from scipy.spatial import cKDTree

from oracle import day_oracle as D
from optimalinterpolation_amd import _lib, day, synthetic

pytestmark = pytest.mark.gpu


def same(a, b):
    ok = np.array_equal(a, b, equal_nan=True)
    if not ok:  # diagnostics for the failure message
        bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
        d = np.abs(a - b)[bad]
        print(f"mismatch: {bad.sum()} entries, max |d| {np.nanmax(d) if d.size else 0}, "
              f"nan-pattern equal {np.array_equal(np.isnan(a), np.isnan(b))}")
    return ok


@pytest.mark.parametrize('std,shape', [(2, (320, 320)), (1, (70, 53)), (2, (17, 40))])
def test_smooth_bit_exact(std, shape):
    rng = np.random.default_rng(std + shape[0])
    f = rng.normal(size=(5,) + shape) * np.array([1e5, 1e5, 3.0, 0.02, 0.01])[:, None, None]
    f = np.abs(f) + np.array([2e5, 2e5, 1.0, 0.001, 0.0005])[:, None, None]
    f[rng.random(f.shape) < 0.45] = np.nan
    f[0, 3, 3] = np.inf
    f[1, 5, 5] = -np.inf
    f[2, 1:, 1:][rng.random(f[2, 1:, 1:].shape) < 0.05] = 50.0  # above vmax
    f[3][:, :] = np.nan                                          # an all-NaN field
    mask = np.where(rng.random(shape) < 0.8, 0.9, np.nan)
    vmax = D.smooth_vmax(300, 9)
    got = _lib.smooth_fields(f, vmax, mask, D.gaussian2d_kernel(std))
    for k in range(5):
        ref = D.smooth(f[k], vmax[k], mask, std)
        assert same(got[k], ref), k


def test_smooth_zero_replacement_bit_exact():
    b = np.full((30, 30), np.nan)
    b[15, 15] = 1.0
    got = day.smooth(b, 5.0, np.ones((30, 30)), 1)
    assert same(got, D.smooth(b, 5.0, np.ones((30, 30)), 1))


def _day(seed=4, nx=64, ice=300e3, obs=700e3, cover=(0.02, 0.18)):
    return synthetic.make_binned_day(seed=seed, nx=nx, ice_radius_m=ice, obs_radius_m=obs, cover=cover)


def test_ball_query_equals_ckdtree():
    d = _day()
    xt, yt, tt, zt = D.training_set(d.sat, d.x, d.y)
    pts = np.column_stack([xt, yt])
    ids = np.where(~np.isnan(d.sie))
    X = np.array([d.x[ids], d.y[ids]]).T
    offs, idx = _lib.ball_query(pts, X, 300e3)
    tree = cKDTree(pts)
    assert offs[0] == 0 and len(idx) == offs[-1]
    for c in range(len(X)):
        ref = np.sort(np.asarray(tree.query_ball_point(x=X[c], r=300e3), dtype=np.int64))
        assert np.array_equal(idx[offs[c]:offs[c + 1]], ref), c
    # gather of those rows, bit-exact
    xyt, zz = _lib.gather_rows(xt, yt, tt, zt, idx)
    assert np.array_equal(xyt, np.stack([xt[idx], yt[idx], tt[idx]], axis=1))
    assert np.array_equal(zz, zt[idx])


def test_ball_query_edges():
    pts = np.array([[0.0, 0.0], [180e3, 240e3], [300e3, 0.0], [300e3 + 1e-6, 0.0], [-300e3, 0.0]])
    offs, idx = _lib.ball_query(pts, np.array([[0.0, 0.0], [5e6, 5e6]]), 300e3)
    assert list(offs) == [0, 4, 4] and list(idx) == [0, 1, 2, 4]
    offs, idx = _lib.ball_query(np.zeros((0, 2)), np.array([[0.0, 0.0]]), 300e3)
    assert list(offs) == [0, 0] and len(idx) == 0
    # more than one chunk of 256 with hits spread over chunks, ascending order
    rng = np.random.default_rng(0)
    p = rng.uniform(-1e6, 1e6, (5000, 2))
    offs, idx = _lib.ball_query(p, np.array([[0.0, 0.0], [9e5, -9e5]]), 3e5)
    for c, q in enumerate([[0.0, 0.0], [9e5, -9e5]]):
        assert np.array_equal(idx[offs[c]:offs[c + 1]], D.ball_query(p, np.array(q), 3e5))


def test_ball_query_many_chunk_batches():
    """More than 256 chunks (the kernels prune chunk boxes 256 at a time):
    index sets and order equal the oracle's on 200 000 points, queries whose
    hits straddle batch boundaries and one that hits nothing."""
    rng = np.random.default_rng(5)
    p = rng.uniform(0.0, 4e6, (200_000, 2))
    p[70_000:70_300] = rng.uniform(1e7, 1.01e7, (300, 2))   # a far-away clump inside batch 1
    q = np.array([[2e6, 2e6], [1.0e7 + 5e3, 1.0e7 + 5e3], [3.9e6, 1e5], [-9e6, -9e6]])
    offs, idx = _lib.ball_query(p, q, 2.5e5)
    for c in range(len(q)):
        assert np.array_equal(idx[offs[c]:offs[c + 1]], D.ball_query(p, q[c], 2.5e5)), c
    assert offs[4] - offs[3] == 0 and offs[2] - offs[1] == 300


def test_pooled_training_set_returns_each_cells_own_rows():
    """bench.py's in-region query: the rank's cells pooled into one training
    set on a lattice; the device query + gather must hand every cell exactly
    its drawn observations, in order (the searched positions are translated
    copies, the gathered columns the drawn values), so the fit equals the
    pre-gathered submission bitwise."""
    import torch
    import bench
    cells = synthetic.make_cells([300, 420, 310, 505, 333], seed=3)
    slices = [cells.subset([0, 1, 2]), cells.subset([3, 4])]
    pool = bench.pool_training_set(slices, synthetic.GRID_M, torch, torch.device('cuda', 0))
    outs = []
    for k, sl in enumerate(slices):
        offs, idx = _lib.ball_query_device(pool['pts'], pool['q'][k], pool['r'])
        assert np.array_equal(offs, sl.offs)
        xyt, z = _lib.gather_rows_device(pool['cols'], idx)
        assert np.array_equal(xyt.cpu().numpy(), sl.xyt) and np.array_equal(z.cpu().numpy(), sl.z)
        a = _lib.gpr_batch_device(xyt, z, sl.offs, sl.xs, sl.mean, x0=bench.X0, opt=True, device=0)
        b = _lib.gpr_batch(sl.xyt, sl.z, sl.offs, sl.xs, sl.mean, x0=bench.X0, opt=True)
        outs.append((a[0], b[0]))
    for a, b in outs:
        assert np.array_equal(a, b)


def test_gather_rejects_bad_index():
    with pytest.raises(_lib.OiError):
        _lib.gather_rows(np.zeros(3), np.zeros(3), np.zeros(3), np.zeros(3), np.array([0, 3]))


def _pass1_rows(d):
    """Plausible pass-1 fields without running the optimiser: hypers varying
    smoothly in space, a few failed (NaN) and out-of-range cells."""
    ids = np.where(~np.isnan(d.sie))
    X = np.array([d.x[ids], d.y[ids]]).T
    u = np.sin(X[:, 0] / 3e5) * np.cos(X[:, 1] / 4e5)
    rows = np.column_stack([0.3 + 0.01 * u, 0.02 + 0.001 * u, -100 + u, 2.5e5 * (1.1 + u),
                            3.0e5 * (1.1 - 0.5 * u), 6.0 + 2 * u, 4e-3 * (1.2 + u),
                            8e-4 * (1.2 - 0.5 * u)])
    rows[3] = np.nan          # a non-PD cell (GPR:187-191)
    rows[5, 3] = 2e6          # above vmax = 600 km (GPR:303)
    return rows


@pytest.mark.parametrize('neighbours', ['device', 'kdtree'])
def test_day_pass2_matches_oracle(neighbours):
    d = _day(seed=7, nx=48, ice=200e3, obs=500e3, cover=(0.02, 0.06))
    rows = _pass1_rows(d)
    res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='20181205', neighbours=neighbours,
                              pass1_rows=rows)
    ref = D.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='20181205', pass1_rows=rows)
    assert set(res) == set(ref)
    for k in day.PASS1_KEYS:
        assert same(res['20181205_' + k], ref['20181205_' + k]), k
    for k in day.HYPER_KEYS:
        assert same(res['20181205_' + k + '_smth'], ref['20181205_' + k + '_smth']), k
    for k in ('interp_smth', 'interp_error_smth'):
        a, b = res['20181205_' + k], ref['20181205_' + k]
        assert np.array_equal(np.isnan(a), np.isnan(b)), k
        ok = ~np.isnan(b)
        assert np.all(np.abs(a[ok] - b[ok]) <= 1e-10 * np.maximum(1.0, np.abs(b[ok]))), k


def test_day_full_fit_runs_and_is_consistent():
    """opt=True end to end on a small day: every ice cell has finite fields, the
    pass-1 fields feed the smoothing exactly as the oracle would smooth them,
    and pass 2 equals the oracle's GPR3D(opt=False) on those smoothed hypers."""
    d = _day(seed=8, nx=40, ice=120e3, obs=450e3, cover=(0.02, 0.05))
    res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d')
    ids = np.where(~np.isnan(d.sie))
    assert np.isfinite(res['d_interp'][ids]).all() and np.isfinite(res['d_interp_smth'][ids]).all()
    rows = np.column_stack([res['d_' + k][ids] for k in day.PASS1_KEYS])
    ref = D.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', pass1_rows=rows)
    for k in day.HYPER_KEYS:
        assert same(res['d_' + k + '_smth'], ref['d_' + k + '_smth']), k
    a, b = res['d_interp_smth'][ids], ref['d_interp_smth'][ids]
    assert np.all(np.abs(a - b) <= 1e-10 * np.maximum(1.0, np.abs(b)))
    assert res.info['evals'][~np.isnan(res.info['evals'])].min() >= 1


def test_day_12p5km_grid_pass2():
    """The 12.5 km configuration (BASELINE config 5): smoothing width std=1
    (GPR:298-302), a 640-wide grid, pass 2 against the oracle."""
    d = synthetic.make_binned_day(seed=9, nx=640, grid_m=12.5e3, ice_radius_m=150e3,
                                  obs_radius_m=460e3, cover=(0.004, 0.012))
    rows = _pass1_rows(d)
    res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', grid_res=12.5,
                              pass1_rows=rows)
    ref = D.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', grid_res=12.5,
                            pass1_rows=rows)
    for k in day.HYPER_KEYS:
        assert same(res['d_' + k + '_smth'], ref['d_' + k + '_smth']), k
    ids = np.where(~np.isnan(d.sie))
    a, b = res['d_interp_smth'][ids], ref['d_interp_smth'][ids]
    assert np.all(np.abs(a - b) <= 1e-10 * np.maximum(1.0, np.abs(b)))


def test_multi_day_batch_equals_day_by_day():
    """interpolate_days fits every day's cells in ONE batched call (days with
    different prior means): per-day results are bitwise those of separate
    interpolate_day calls (cells are independent; the mean is folded exactly)."""
    days = []
    for k in range(3):
        d = _day(seed=20 + k, nx=40, ice=110e3, obs=450e3, cover=(0.02, 0.05))
        days.append((d, 0.27 + 0.01 * k, '2018120%d' % k))
    batched = day.interpolate_days([(d.sat, d.sie, m, dt) for d, m, dt in days], days[0][0].x,
                                   days[0][0].y)
    for (d, m, dt), res in zip(days, batched):
        one = day.interpolate_day(d.sat, d.sie, d.x, d.y, m, date=dt)
        assert set(res) == set(one)
        for key in one:
            assert same(res[key], one[key]), key
        ids = np.where(~np.isnan(d.sie))
        assert np.isfinite(res[dt + '_interp_smth'][ids]).all()
