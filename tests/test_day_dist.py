"""Multi-rank plumbing of the day pipeline (day.interpolate_day)
with the gloo backend on CPU, world_size 2: partition of the cells, the one
all_gather of pass-1 rows, local smoothing on every rank, the final gather.
The liboi device calls are replaced by CPU stand-ins built from the oracle
(the GPU path itself is covered by tests/test_gpu_day.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeLib:
    """CPU stand-ins with liboi's signatures (oracle-backed, deterministic)."""

    @staticmethod
    def ball_query_device(pts, q, r, counts_only=False, **kw):
        from oracle import day_oracle as D
        P, Q = pts.numpy(), q.numpy()
        ids = [D.ball_query(P, Q[k], r) for k in range(len(Q))]
        offs = np.zeros(len(Q) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(i) for i in ids])
        if counts_only:
            return offs, None
        import torch
        return offs, torch.from_numpy(np.concatenate(ids) if ids else np.zeros(0, np.int64))

    @staticmethod
    def gather_rows_device(cols, idx, **kw):
        import torch
        i = idx.numpy()
        x, y, t, z = (c.numpy() for c in cols)
        return torch.from_numpy(np.stack([x[i], y[i], t[i]], axis=1)), torch.from_numpy(z[i])

    @staticmethod
    def gpr_batch_device(xyt, z, offs, xs, mean, x0=None, opt=True, hyp=None, info=False, **kw):
        from oracle import gp_oracle as O
        X, Z = xyt.numpy(), z.numpy()
        out = np.zeros((len(offs) - 1, 8))
        for c in range(len(offs) - 1):
            a, b = offs[c], offs[c + 1]
            h = (2.5e5, 2.5e5, 5.0, 4e-3, 1e-3) if opt else tuple(hyp[c])
            fs, sd, lZ = O.predict(X[a:b], Z[a:b], xs[c:c + 1], mean, h[:3], h[3], h[4])
            out[c] = [fs[0], sd[0], lZ, *h]
        return out, np.zeros(len(out), np.int32), np.ones((len(out), 4), np.int32)

    @staticmethod
    def smooth_fields(fields, vmax, mask, kern, **kw):
        from oracle import day_oracle as D
        std = {9: 1, 17: 2}[kern.shape[0]]
        return np.stack([D.smooth(f, v, mask, std) for f, v in zip(fields, vmax)])


def _day():
    from optimalinterpolation_amd import synthetic
    return synthetic.make_binned_day(seed=5, nx=36, ice_radius_m=110e3, obs_radius_m=420e3,
                                     cover=(0.01, 0.02))


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from optimalinterpolation_amd import day
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    day._lib = FakeLib()
    d = _day()
    res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', rank=rank, world=world,
                              device='cpu')
    q.put((rank, None if res is None else {k: v for k, v in res.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.blas_default
def test_day_two_ranks_equals_one():
    from optimalinterpolation_amd import day
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[1] is None and got[0] is not None
    saved = day._lib
    try:
        day._lib = FakeLib()
        d = _day()
        ref = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', device='cpu')
    finally:
        day._lib = saved
    assert set(got[0]) == set(ref)
    for k in ref:
        assert np.array_equal(got[0][k], ref[k], equal_nan=True), k


def test_day_no_ice_cells():
    """A day whose ice mask is empty (GPR:248 IDs empty): every field NaN, no error."""
    from optimalinterpolation_amd import day
    saved = day._lib
    try:
        day._lib = FakeLib()
        d = _day()
        sie = np.full(d.sie.shape, np.nan)
        res = day.interpolate_day(d.sat, sie, d.x, d.y, d.mean, date='d', device='cpu')
    finally:
        day._lib = saved
    assert res.info['ncell'] == 0
    for k, v in res.items():
        assert v.shape == sie.shape and np.isnan(v).all(), k


def _empty_worker(rank, world, port, q):
    import torch.distributed as dist
    from optimalinterpolation_amd import day
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    day._lib = FakeLib()
    d = _day()
    sie = np.full(d.sie.shape, np.nan)
    res = day.interpolate_day(d.sat, sie, d.x, d.y, d.mean, date='d', rank=rank, world=world,
                              device='cpu')
    q.put((rank, None if res is None else bool(all(np.isnan(v).all() for v in res.values()))))
    dist.barrier()
    dist.destroy_process_group()


def test_day_two_ranks_no_ice():
    """Both collectives are skipped consistently when no rank has a cell."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0] is True and got[1] is None
