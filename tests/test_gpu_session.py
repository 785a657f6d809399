"""The continuous-batching session (oi_session_*, include/oi.h) on the GPU.

A stream of batches through one session must give, cell for cell, bitwise
the results of one oi_gpr_batch call over the same cells (per-cell arithmetic
never depends on which cells share a round), for fits (GPR3D opt=True,
GPR:143-191) and predict-only batches (opt=False, GPR:170-182), with host and
device inputs, whatever the order of submit / wait calls.
"""
import numpy as np
import pytest

from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib, synthetic

pytestmark = pytest.mark.gpu

X0 = np.array(O.X0_PRODUCTION)


def _slices(cells, k):
    edges = np.linspace(0, cells.ncell, k + 1).astype(int)
    return [cells.subset(np.arange(a, b)) for a, b in zip(edges[:-1], edges[1:])]


def test_session_fit_equals_one_call():
    cells = synthetic.make_cells([0, 1, 40, 70, 130, 200, 64, 65, 333, 90, 17, 250], seed=41)
    ref, rst, rinf = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True,
                                    info=True)
    parts = _slices(cells, 4)
    with _lib.Session() as s:
        tickets = [s.submit(p.xyt, p.z, p.offs, p.xs, p.mean, x0=X0) for p in parts]
        # wait out of order: the last batch first, then the rest
        res = {3: s.wait(tickets[3])}
        for k in (1, 0, 2):
            res[k] = s.wait(tickets[k])
    out = np.concatenate([res[k][0] for k in range(4)])
    st = np.concatenate([res[k][1] for k in range(4)])
    inf = np.concatenate([res[k][2] for k in range(4)])
    assert np.array_equal(out, ref, equal_nan=True)
    assert np.array_equal(st, rst)
    assert np.array_equal(inf, rinf)


def test_session_pipelined_device_inputs():
    import torch
    cells = synthetic.make_cells(np.random.default_rng(5).integers(50, 400, 24), seed=43)
    ref, _, rinf = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True,
                                  info=True)
    parts = _slices(cells, 6)
    dev = [(torch.from_numpy(p.xyt).cuda(), torch.from_numpy(p.z).cuda()) for p in parts]
    outs = {}
    with _lib.Session(device_inputs=True, profile=True) as s:
        t = []
        for k, p in enumerate(parts):  # the bench's depth-1 pipeline
            t.append(s.submit(dev[k][0], dev[k][1], p.offs, p.xs, p.mean, x0=X0))
            if k >= 1:
                outs[k - 1] = s.wait(t[k - 1])
        outs[len(parts) - 1] = s.wait(t[-1])
        assert all(s.done(x) for x in t)
    out = np.concatenate([outs[k][0] for k in range(len(parts))])
    inf = np.concatenate([outs[k][2] for k in range(len(parts))])
    assert np.array_equal(out, ref)
    assert np.array_equal(inf, rinf)


def test_session_predict_and_fit_mixed():
    cells = synthetic.make_cells([100, 260, 30, 500, 0, 75], seed=47)
    hyp = np.tile(synthetic.FIXED_HYPERS, (cells.ncell, 1))
    rp, _, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
    rf, _, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True)
    with _lib.Session() as s:
        a = s.submit(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
        b = s.submit(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0)
        e = s.submit(np.zeros((0, 3)), np.zeros(0), [0], np.zeros((0, 3)), cells.mean, x0=X0)
        assert s.done(e)  # an empty batch completes at once
        pb = s.wait(b)
        pa = s.wait(a)
        s.wait(-1)
    assert np.array_equal(pa[0], rp, equal_nan=True)
    assert np.array_equal(pb[0], rf, equal_nan=True)
    for k in range(cells.ncell):  # T1 against the oracle (GPR:173-182)
        x, y, xs = cells.cell(k)
        if len(y) == 0:
            continue
        fs, sd, lZ = O.predict(x, y, xs, cells.mean, synthetic.FIXED_HYPERS[:3], synthetic.FIXED_HYPERS[3],
                               synthetic.FIXED_HYPERS[4])
        assert abs(pa[0][k, 0] - fs[0]) <= 1e-10 * max(1, abs(fs[0]))
        assert abs(pa[0][k, 1] - sd[0]) <= 1e-10 * max(1, abs(sd[0]))


def test_device_input_checks():
    import torch
    cells = synthetic.make_cells([20], seed=1)
    with pytest.raises(ValueError, match='float64'):
        _lib.gpr_batch_device(torch.from_numpy(cells.xyt).float().cuda(), torch.from_numpy(cells.z).cuda(),
                              cells.offs, cells.xs, cells.mean, x0=X0)
    with pytest.raises(ValueError, match='cuda'):
        _lib.gpr_batch_device(torch.from_numpy(cells.xyt), torch.from_numpy(cells.z).cuda(),
                              cells.offs, cells.xs, cells.mean, x0=X0)


def test_session_wait_all_keeps_results():
    """wait(-1) drains everything and hands back every uncollected ticket's
    results; they can still be collected one by one afterwards, once."""
    cells = synthetic.make_cells([80, 150, 40, 210], seed=53)
    hyp = np.tile(synthetic.FIXED_HYPERS, (cells.ncell, 1))
    ref, _, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
    parts = _slices(cells, 2)
    with _lib.Session() as s:
        t = [s.submit(p.xyt, p.z, p.offs, p.xs, p.mean, opt=False,
                      hyp=np.tile(synthetic.FIXED_HYPERS, (p.ncell, 1))) for p in parts]
        got0 = s.wait(t[0])
        allres = s.wait(-1)
        assert set(allres) == {t[1]}
        got1 = s.wait(t[1])
        assert got1[0] is allres[t[1]][0]
        with pytest.raises(KeyError):
            s.wait(t[1])   # already collected
        with pytest.raises(KeyError):
            s.wait(t[0])
    assert np.array_equal(np.concatenate([got0[0], got1[0]]), ref)


def test_session_device_inputs_from_side_stream():
    """A producer on a non-default torch stream: each submit is ordered after
    the stream current AT SUBMIT (oi_session_set_stream), not the one current
    when the session was created."""
    import torch
    cells = synthetic.make_cells([300, 120, 450], seed=59)
    hyp = np.tile(synthetic.FIXED_HYPERS, (cells.ncell, 1))
    ref, _, _ = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
    xh = torch.from_numpy(cells.xyt).pin_memory()
    zh = torch.from_numpy(cells.z).pin_memory()
    side = torch.cuda.Stream()
    with _lib.Session(device_inputs=True) as s:
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)             # keep the producer stream busy
            xd = torch.empty_like(xh, device='cuda')
            zd = torch.empty_like(zh, device='cuda')
            xd.copy_(xh, non_blocking=True)
            zd.copy_(zh, non_blocking=True)
            t = s.submit(xd, zd, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
        out, st, _ = s.wait(t)
    assert np.array_equal(out, ref)


def test_tiny_pool_nomem_then_normal_call():
    """A batch whose inputs do not fit the arena (they go to a private
    buffer) and whose cell exceeds it: OI_E_NOMEM, and the arena stays
    consistent -- the next call with the same pool is bitwise the default's
    (oi_engine.cpp Engine::submit)."""
    rng = np.random.default_rng(61)
    ncell, n = 200, 1500                         # 300 k obs: ~22 MB of inputs > 16 MB pool
    xyt = np.column_stack([rng.uniform(0, 5e5, ncell * n), rng.uniform(0, 5e5, ncell * n),
                           rng.integers(0, 9, ncell * n).astype(float)])
    z = rng.normal(0.3, 0.05, ncell * n)
    offs = np.arange(ncell + 1, dtype=np.int64) * n
    xs = np.tile([2.5e5, 2.5e5, 4.0], (ncell, 1))
    pool = 16 << 20
    with pytest.raises(_lib.OiError, match='-3'):
        _lib.gpr_batch(xyt, z, offs, xs, 0.28, x0=X0, opt=True, pool_bytes=pool)
    small = synthetic.make_cells([90, 30, 150, 60], seed=67)
    hyp = np.tile(synthetic.FIXED_HYPERS, (small.ncell, 1))
    for _ in range(3):
        got, st, _ = _lib.gpr_batch(small.xyt, small.z, small.offs, small.xs, small.mean, opt=False, hyp=hyp,
                                    pool_bytes=pool)
        assert np.all(st == 0)
    ref, _, _ = _lib.gpr_batch(small.xyt, small.z, small.offs, small.xs, small.mean, opt=False, hyp=hyp)
    assert np.array_equal(got, ref)


def test_session_unprofiled_groups_equal_profiled(monkeypatch):
    """the unprofiled session completes rounds through the host flag
    k_finalize writes into pinned memory (no stream synchronise), profiled
    rounds synchronise instead.  With two stream groups (OI_GROUPS=2) and a
    stream of small batches -- including batches whose cells are all n = 0 or
    n = 1 (rounds with nothing to factor) -- both completion paths give the same
    outputs, status and CG info bit for bit, and the round counter advances."""
    monkeypatch.setenv('OI_GROUPS', '2')
    rng = np.random.default_rng(77)
    batches = []
    for k in range(14):
        if k in (3, 9):
            sizes = [0, 0, 1]
        else:
            sizes = rng.integers(20, 260, int(rng.integers(1, 5)))
        batches.append(synthetic.make_cells(sizes, seed=500 + k))
    res = {}
    for prof in (False, True):
        _lib.profile_reset()
        outs = []
        with _lib.Session(profile=prof) as s:
            t = [s.submit(b.xyt, b.z, b.offs, b.xs, b.mean, x0=X0) for b in batches]
            for k, tk in enumerate(t):
                outs.append(s.wait(tk))
        res[prof] = outs
        assert _lib.profile_json()['rounds'] > 0, prof
    for a, b in zip(res[False], res[True]):
        assert np.array_equal(a[0], b[0], equal_nan=True)
        assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
