"""The GPU objective's distance to the reference against the reference's own
rounding noise (VERDICT r5 "next" item 1), on the bench-day cells of
tests/golden/day_ref_fits.npz: the 360 cells the thresholds below were set on
and, separately, the 320-cell replication sample appended in round 6
(stratum 3), on which the same thresholds are asserted unchanged.

Fixture tests/golden/day_ref_t1.npz (tests/golden/make_day_t1.py): the
reference's own SMLII (GPR_CS2S3.py:107-141) on each cell in the 5
observation orders of its fits, at x0 (GPR:217) and at the hypers its run 0
ended at.  Per cell, point and quantity q (nlZ, dnlZ[0..4]):

    d_gpu = |GPU(order 0) - ref(order 0)|,   d_ref = max_k |ref(order k) - ref(order 0)|

d_ref is how far the reference itself moves when only the summation order of
its observations changes (the CG's stopping point is chaotic
in exactly that noise).  If the GPU were "one more observation order",
d_gpu would be distributed like ONE of the four |ref_k - ref_0|, so its median
ratio to their max is below 1; the test asserts the median ratio <= 2 per
quantity at the fitted hypers, for both site forms, and prints the
distribution (both distances floored at one rounding unit eps |ref_0|); at
x0, where every value is decided in its last bit, the GPU's median distance
is asserted to be <= 4 rounding units.
OI_T1_DUMP=dir saves the arrays."""
import os

import numpy as np
import pytest

from conftest import load_golden
from optimalinterpolation_amd import _lib

pytestmark = pytest.mark.gpu
QNAMES = ['nlZ', 'g_lx', 'g_ly', 'g_lt', 'g_sf2', 'g_sn2']
_CACHE = {}


def gpu_values(dedup):
    if dedup not in _CACHE:
        fx, t1 = load_golden('day_ref_fits.npz'), load_golden('day_ref_t1.npz')
        assert np.array_equal(fx['cells'][:len(t1['cells'])], t1['cells'])
        fx = {k: fx[k] for k in fx}
        nc = len(t1['cells'])
        fx['offs'] = fx['offs'][:nc + 1]
        fx['x'] = fx['x'].reshape(-1, 3)[:fx['offs'][-1]]
        fx['y'] = fx['y'][:fx['offs'][-1]]
        x, y, offs, mean = fx['x'].reshape(-1, 3), fx['y'], fx['offs'], float(fx['mean'])
        old = os.environ.get('OI_DEDUP')
        os.environ['OI_DEDUP'] = str(dedup)
        try:
            vals = np.full((len(offs) - 1, 2, 6), np.nan)
            for p in range(2):
                h = t1['hyp'][:, p].copy()
                ok = np.isfinite(h).all(1)
                h[~ok] = t1['hyp'][~ok, 0]
                nlz, g, st = _lib.nlml_grad_batch(x, y, np.full(len(y), mean), offs, h)
                vals[:, p, 0] = nlz
                vals[:, p, 1:] = g[:, :5]
                vals[~ok | (st != 0), p] = np.nan
        finally:
            if old is None:
                del os.environ['OI_DEDUP']
            else:
                os.environ['OI_DEDUP'] = old
        ref = np.concatenate([t1['nlz'][..., None], t1['grad'][..., :5]], -1)  # cell, point, order, q
        if os.environ.get('OI_T1_DUMP'):
            os.makedirs(os.environ['OI_T1_DUMP'], exist_ok=True)
            np.savez(os.path.join(os.environ['OI_T1_DUMP'], f'gpu_day_t1_dedup{dedup}.npz'), gpu=vals, ref=ref,
                     sizes=t1['sizes'])
        _CACHE[dedup] = (vals, ref, t1['sizes'], fx['stratum'][:len(t1['cells'])])
    return _CACHE[dedup]


def distances(dedup):
    vals, ref, sizes, _ = gpu_values(dedup)
    d_gpu = np.abs(vals - ref[:, :, 0])                                  # cell, point, q
    d_ref = np.max(np.abs(ref[:, :, 1:] - ref[:, :, :1]), axis=2)        # cell, point, q
    return d_gpu, d_ref, sizes


@pytest.mark.parametrize('dedup', [1, 0])
def test_gpu_objective_within_reference_order_noise(dedup):
    """At the hypers the reference's fits ended at (point 'fit', where the
    chaotic stop is decided) the GPU's distance to run 0 is asserted against
    the reference's own order spread: median ratio <= 2 for nlZ and every
    gradient component (round 6, both site forms: 0.55 .. 0.68, i.e. inside
    the spread).  At x0 (l = 25 km, sf2 = sn2 = 1) every value is decided in
    its last bit: the reference's orders often agree bit for bit there (np.trace
    and numpy's pairwise sums barely move with the order: median 0.5 - 2.1
    units eps |v| over the quantities), so the ratio is one of ulps; asserted as
    median d_gpu <= 4 units (measured, round 6, OI_DEDUP=1: 0 - 1.2 units on
    nlZ and the length-scale gradients, 3.0 on dnlZ[3] and 2.3 on dnlZ[4] --
    the threshold was set after seeing these; an extended-precision check of
    12 cells puts both the GPU and the reference within ~1 ulp of the exact
    value there)."""
    d_gpu, d_ref, sizes = distances(dedup)
    vals, ref, _, stratum = gpu_values(dedup)
    # floor: one unit of rounding of the value itself -- at x0 (l = 25 km) the
    # reference's nlZ often does not move at all with the order
    ulp = np.finfo(float).eps * np.maximum(np.abs(ref[:, :, 0]), np.finfo(float).tiny)
    ratio = np.maximum(d_gpu, ulp) / np.maximum(d_ref, ulp)
    bad = []
    samples = [('base', stratum != 3)] + ([('replication', stratum == 3)] if np.any(stratum == 3) else [])
    for sname, m in samples:
        for p, pname in enumerate(('x0', 'fit')):
            for q, qn in enumerate(QNAMES):
                ok = np.isfinite(ratio[:, p, q]) & m
                r = ratio[ok, p, q]
                big = sizes[ok] >= 600
                med = float(np.median(r))
                ulps = float(np.median(d_gpu[ok, p, q] / ulp[ok, p, q]))
                ulps_ref = float(np.median(d_ref[ok, p, q] / ulp[ok, p, q]))
                print(f"OI_DEDUP={dedup} {sname:11s} {pname:3s} {qn:6s}: d_gpu/d_ref median {med:.3f} "
                      f"[q25 {np.quantile(r, .25):.3f}, q75 {np.quantile(r, .75):.3f}, q90 {np.quantile(r, .9):.3f}], "
                      f"n>=600 median {np.median(r[big]) if big.any() else np.nan:.3f}, > 1 in {np.mean(r > 1):.3f}; "
                      f"median d_ref {np.median(d_ref[ok, p, q]):.2e} ({ulps_ref:.2f} ulp), "
                      f"d_gpu {np.median(d_gpu[ok, p, q]):.2e} ({ulps:.2f} ulp) ({len(r)} cells)")
                if pname == 'fit' and med > 2.0:
                    bad.append((sname, pname, qn, 'ratio', med))
                if pname == 'x0' and ulps > 4.0:
                    bad.append((sname, pname, qn, 'ulps', ulps))
    assert not bad, bad
