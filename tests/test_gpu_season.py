"""Config 5 on the GPU: a 64-cell slice of
one GPU's share of the 12.5 km season day -- the 640 x 640 grid's cells inside
the disc, n ~ U{300..5000}, observations snapped to the 12.5 km lattice,
x0 of GPR_CS2S3.py:217 at grid_res = 12.5, LPT-split into 8 shares as
`bench.py --workload season` does -- fitted through a session (GPR3D
opt=True, GPR:143-191) in four batches, and T1 checked against
the CPU oracle on 4 of its cells at the hypers the GPU found: SMLII nlZ and
gradient (GPR:107-141) and the predict block fs / sd / lZ (GPR:173-182)
within 1e-10."""
import numpy as np
import pytest

from oracle import gp_oracle as O
from test_gpu_parity import grad_scale
from optimalinterpolation_amd import _lib, driver, synthetic

pytestmark = pytest.mark.gpu

X0_12P5 = np.array([np.log(12.5e3), np.log(12.5e3), 0.0, 0.0, 0.0, np.log(.1)])  # GPR:217, grid_res = 12.5
RTOL = 1e-10


def season_slice(ncell=64, share=0, shares=8):
    cen, sizes = synthetic.season_day_plan(seed=0)
    est = driver.expected_sites(sizes, grid_m=synthetic.GRID_12P5_M)
    parts = driver.lpt_partition(driver.cell_costs(sizes, sites=est), shares)
    mine = np.asarray(parts[share])
    pick = mine[np.argsort(sizes[mine], kind='stable')][np.linspace(0, len(mine) - 1, ncell).astype(int)]
    return synthetic.season_cells(cen, sizes, pick, seed=0)


def test_season_slice_fit_and_t1():
    cells = season_slice()
    n = cells.sizes
    assert n.max() > 4500 and n.min() < 600
    edges = np.linspace(0, cells.ncell, 5).astype(int)
    parts = [cells.subset(np.arange(a, b)) for a, b in zip(edges[:-1], edges[1:])]
    with _lib.Session() as s:
        tick = [s.submit(p.xyt, p.z, p.offs, p.xs, p.mean, x0=X0_12P5) for p in parts]
        res = [s.wait(t) for t in tick]
    out = np.concatenate([r[0] for r in res])
    status = np.concatenate([r[1] for r in res])
    info = np.concatenate([r[2] for r in res])
    assert np.all(status == 0) and np.isfinite(out).all()
    print(f"season slice: {cells.ncell} cells, n {n.min()}..{n.max()}, "
          f"{info[:, 3].mean():.1f} evaluations per cell")
    # T1 on 4 cells spread over n
    for c in np.argsort(n)[[5, 25, 45, 58]]:
        x, z, xs = cells.cell(int(c))
        hyp = out[c, 3:8]
        h = np.r_[np.log(hyp), np.log(.1)]
        mX = np.full(len(z), cells.mean)
        f_cpu, g_cpu = O.neg_log_ml(h, x, z, mX)
        nlz, grad, st = _lib.nlml_grad_batch(x, z, mX, np.array([0, len(z)]), h[None, :])
        f_cpu = float(np.asarray(f_cpu).ravel()[0])
        g_cpu = np.asarray(g_cpu, float).ravel()
        assert st[0] == 0
        assert abs(nlz[0] - f_cpu) <= RTOL * max(1.0, abs(f_cpu)), (c, nlz[0], f_cpu)
        gs = np.abs(g_cpu) + grad_scale(h, x, z, mX)  # tests/test_gpu_parity.py's T1 rule
        assert np.all(np.abs(grad[0] - g_cpu) <= RTOL * gs), (c, grad[0], g_cpu)
        fs, sd, lz = O.predict(x, z, xs, cells.mean, hyp[:3], hyp[3], hyp[4])
        for gpu, ref in ((out[c, 0], fs), (out[c, 1], sd), (out[c, 2], lz)):
            ref = float(np.ravel(ref)[0])
            assert abs(gpu - ref) <= RTOL * max(1.0, abs(ref)), (c, gpu, ref)
        print(f"  cell n={len(z)}: nlZ {nlz[0]:.10e} (oracle {f_cpu:.10e}), fs {out[c, 0]:.12f}")
