"""bench.py's pooled training set (the radius query and gather of GPR:159-161
inside the day bench's timed region), checked on the CPU with the oracle's
ball query (oracle/day_oracle.py, cKDTree's distance test): every cell's query
returns exactly its own observations, in drawn order, and the gathered columns
are the drawn values."""
import numpy as np
import torch

import bench
from oracle import day_oracle as D
from optimalinterpolation_amd import synthetic


def test_pool_queries_return_each_cells_own_rows():
    day = synthetic.make_day(seed=2, max_cells=300)
    slices = [day.subset(np.arange(0, 130)), day.subset(np.arange(130, 300))]
    pool = bench.pool_training_set(slices, synthetic.GRID_M, torch, torch.device('cpu'))
    pts = pool['pts'].numpy()
    cols = [c.numpy() for c in pool['cols']]
    assert pool['M'] == len(day.z) == len(pts)
    base = 0
    for k, sl in enumerate(slices):
        q = pool['q'][k].numpy()
        for c in range(sl.ncell):
            idx = D.ball_query(pts, q[c], pool['r'])
            a, b = sl.offs[c], sl.offs[c + 1]
            assert np.array_equal(idx, np.arange(base + a, base + b)), (k, c)
            assert np.array_equal(np.column_stack([cols[0][idx], cols[1][idx], cols[2][idx]]), sl.xyt[a:b])
            assert np.array_equal(cols[3][idx], sl.z[a:b])
        base += sl.offs[-1]


def test_pool_radius_covers_snapped_observations():
    # observations lie within RADIUS_M of the centre before snapping to the grid,
    # so within RADIUS_M + grid / sqrt(2) after: the query radius has room
    rng = np.random.default_rng(0)
    x, _ = synthetic.cell_obs(rng, 4e6, 4e6, 20000)
    d = np.hypot(x[:, 0] - 4e6, x[:, 1] - 4e6)
    assert d.max() <= synthetic.RADIUS_M + synthetic.GRID_M / np.sqrt(2) + 1e-6
    assert bench.POOL_PITCH_M > 2 * (synthetic.RADIUS_M + synthetic.GRID_M)


def test_cpu_baseline_evaluations_come_from_the_reference_on_this_day():
    """cpu_baseline's E(n): the reference's own evaluation
    counts on the bench day's cells (tests/golden/day_ref_fits.npz, per 300-wide
    n bucket), not a fit to other cells: every bucket value is the fixture's
    own bucket mean over its cells and 5 observation orders, and the day-weighted
    mean is their average."""
    d = np.load('tests/golden/day_ref_fits.npz')
    E, desc, e_fix = bench.reference_evals_model()
    sizes, ev = d['sizes'], d['evals'].astype(float)
    means = []
    for lo in range(300, 3000, 300):
        m = (sizes >= lo) & (sizes < (lo + 300 if lo < 2700 else 3001))
        assert m.sum() >= 8
        means.append(ev[m].mean())
        assert np.allclose(E(np.array([lo, lo + 150, lo + 299])), ev[m].mean()), lo
    assert abs(e_fix - np.mean(means)) < 1e-9 and 'day_ref_fits.npz' in desc
    assert np.all(np.isfinite(E(np.array([3500.0, 5000.0]))))
