"""CPU checks of the day-level restatements (oracle/day_oracle.py) and of the
host-side pieces of the day pipeline (optimalinterpolation_amd/day.py).

Pinning: numpy's summation order and ``np.nanmean`` are pinned bit-for-bit to
numpy itself; the neighbour query to scipy's cKDTree (the reference's own
call, GPR:159); the training-set assembly to a literal restatement of
GPR:223-246.  The astropy convolution used by ``smooth`` (GPR:73) cannot be
pinned (astropy is absent, the reference pins no version): it is checked
against an independent scipy.ndimage formulation of the same definition
(parity unpinned against astropy itself)."""
import os
import pickle

import numpy as np
import pytest
from scipy import ndimage
from scipy.spatial import cKDTree

from oracle import day_oracle as D
from optimalinterpolation_amd import day, synthetic


@pytest.mark.parametrize('n', [0, 1, 7, 8, 9, 127, 128, 129, 136, 1000, 8191, 8192, 8193, 20000, 102400])
def test_numpy_summation_order(n):
    rng = np.random.default_rng(n)
    a = rng.normal(size=n) * rng.choice([1.0, 1e8, 1e-8], size=n)
    assert D.numpy_pairwise_sum(a) == np.sum(a)


def test_nanmean_order():
    rng = np.random.default_rng(5)
    a = rng.normal(size=(320, 320)) * 1e3
    a[rng.random(a.shape) < 0.4] = np.nan
    ok = ~np.isnan(a)
    assert D.numpy_pairwise_sum(np.where(ok, a, 0.0)) / ok.sum() == np.nanmean(a)


def test_training_set_matches_restatement():
    d = synthetic.make_binned_day(seed=3, nx=64, ice_radius_m=300e3, obs_radius_m=600e3)
    for a, b in zip(day.training_set(d.sat, d.x, d.y), D.training_set(d.sat, d.x, d.y)):
        assert np.array_equal(a, b)


def test_ball_query_oracle_equals_ckdtree_sets():
    d = synthetic.make_binned_day(seed=4, nx=64, ice_radius_m=300e3, obs_radius_m=700e3)
    xt, yt, _, _ = D.training_set(d.sat, d.x, d.y)
    pts = np.column_stack([xt, yt])
    tree = cKDTree(pts)
    ids = np.where(~np.isnan(d.sie))
    X = np.array([d.x[ids], d.y[ids]]).T
    for q in X[::7]:
        ref = np.sort(np.asarray(tree.query_ball_point(x=q, r=300e3), dtype=np.int64))
        assert np.array_equal(D.ball_query(pts, q, 300e3), ref)
    # lattice points exactly at the radius (3-4-5 triangle: 180 km, 240 km) are inside
    edge = np.array([[0.0, 0.0], [180e3, 240e3], [300e3, 0.0], [300e3 + 1e-6, 0.0]])
    assert list(D.ball_query(edge, np.array([0.0, 0.0]), 300e3)) == [0, 1, 2]
    assert sorted(cKDTree(edge).query_ball_point([0.0, 0.0], 300e3)) == [0, 1, 2]


def test_gaussian_kernel_shape_and_mass():
    for std, size in ((1, 9), (2, 17), (1.5, 13)):
        k = D.gaussian2d_kernel(std)
        assert k.shape == (size, size)
        assert abs(k.sum() - 1.0) < 1e-15
        assert np.array_equal(k, k[::-1, ::-1]) and np.array_equal(k, k.T)
        assert np.array_equal(day.gaussian2d_kernel(std), k)


def _ndimage_convolve(data, k):
    """Independent formulation: sum(v k) / sum(k over valid), fill 0 valid."""
    valid = ~np.isnan(data)
    top = ndimage.correlate(np.where(valid, data, 0.0), k[::-1, ::-1], mode='constant', cval=0.0)
    bot = ndimage.correlate(valid.astype(float), k[::-1, ::-1], mode='constant', cval=1.0)
    with np.errstate(invalid='ignore', divide='ignore'):
        return np.where(bot <= 1e-300, np.nan, top / bot)


@pytest.mark.parametrize('std', [1, 2])
def test_convolution_restatement_vs_ndimage(std):
    rng = np.random.default_rng(std)
    a = rng.normal(size=(70, 53)) + 3.0
    a[rng.random(a.shape) < 0.5] = np.nan
    a[30:60, 20:50] = np.nan  # a NaN block larger than the kernel -> NaN output inside
    k = D.gaussian2d_kernel(std)
    got = D.convolve_interpolate(a, k)
    ref = _ndimage_convolve(a, k)
    both = np.isnan(got) & np.isnan(ref)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.allclose(got[~both], ref[~both], rtol=1e-13, atol=0)
    assert np.isnan(got[45, 35])
    a[:20, :20] = np.nan      # padding is a valid 0 (boundary='fill'): corner -> 0
    assert D.convolve_interpolate(a, k)[0, 0] == 0.0


def test_smooth_edge_semantics():
    k = 2
    a = np.full((40, 40), np.nan)
    a[10:30, 10:30] = 0.5
    a[15, 15] = np.inf        # inf -> NaN (GPR:71)
    a[20, 20] = 10.0          # clipped to vmax (GPR:72)
    mask = np.full((40, 40), np.nan)
    mask[12:28, 12:28] = 1.0
    s = D.smooth(a, 1.0, mask, k)
    assert np.isnan(s[0, 0]) and np.isnan(s[13, 30])            # outside the mask
    assert np.all(np.isfinite(s[12:28, 12:28]))
    assert s[20, 20] < 1.0                                       # clip happened before smoothing
    # a window with only padding + NaN gives 0 -> replaced by the nanmean
    b = np.full((30, 30), np.nan)
    b[15, 15] = 1.0
    m = np.ones((30, 30))
    sb = D.smooth(b, 5.0, m, 1)
    conv = D.convolve_interpolate(b, D.gaussian2d_kernel(1))
    assert conv[0, 0] == 0.0 and sb[0, 0] == np.nanmean(conv)  # zeros -> nanmean (GPR:74)
    assert np.isnan(sb[8, 8])                                  # all-NaN window, no padding


def test_readfb_and_save_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    dates = ['20181130', '20181201', '20181202']
    for name in ('CS2_SAR', 'CS2_SARIN', 'S3A', 'S3B'):
        dd = {dt: rng.normal(size=(8, 8)) for dt in dates}
        if name == 'S3B':
            dd.pop('20181130')  # dates missing from a satellite are dropped (GPR:57)
        with open(tmp_path / f'{name}_dailyFB_25km_2018-2019_season.pkl', 'wb') as f:
            pickle.dump(dd, f, protocol=2)
    sie = {dt: rng.random((8, 8)) for dt in dates}
    with open(tmp_path / 'SIE_masking_25km_2018-2019_season.pkl', 'wb') as f:
        pickle.dump(sie, f, protocol=2)
    obs, mask, dt = day.readFB(str(tmp_path), 25, '2018-2019')
    assert dt == ['20181201', '20181202'] and obs.shape == (8, 8, 4, 2) and mask.shape == (8, 8, 2)
    assert np.isnan(mask[sie['20181201'] < 0.15, 0]).all()
    res = {'20181201_interp': obs[:, :, 0, 0]}
    day.save(res, str(tmp_path / 'out.pkl'))
    back = day._load_pickle(str(tmp_path / 'out.pkl'))
    assert np.array_equal(back['20181201_interp'], res['20181201_interp'])


def test_safe_unpickler_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ('true',))
    p = tmp_path / 'evil.pkl'
    with open(p, 'wb') as f:
        pickle.dump({'a': Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        day._load_pickle(str(p))


def test_quicklook_writer(tmp_path):
    from scipy.io import netcdf_file
    fs = np.arange(12.0).reshape(3, 4)
    p = str(tmp_path / 'q.nc')
    day.write_quicklook(p, fs, fs * 0.1, lat=fs + 60, lon=fs - 10, fmt='netcdf3')
    with netcdf_file(p, 'r', mmap=False) as f:
        assert np.array_equal(f.variables['radar_freeboard'][:], fs)
        assert set(f.variables) == {'lat', 'lon', 'radar_freeboard', 'uncertainty'}
