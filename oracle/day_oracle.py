"""CPU oracle for the day-level pipeline around the per-cell GP -- TEST
INFRASTRUCTURE ONLY (same rules as ``gp_oracle.py``: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it; the
product package never imports it).

Restates, from ``2021_paper_production/GPR_CS2S3.py`` (``GPR:``):

* ``training_set``   <- GPR:223-246 (flatten 4 satellites x T days of binned
                        grids into x_train, y_train, t_train, z)
* ``ball_query``     <- ``X_tree.query_ball_point(X[index], r=radius*1000)``
                        GPR:159 (scipy cKDTree), returned SORTED (the tree's own
                        order depends on its build; see ``ball_query``)
* ``gaussian2d_kernel``, ``convolve_interpolate``
                     <- astropy ``Gaussian2DKernel(x_stddev=std, y_stddev=std)``
                        and ``convolve(...)`` with its defaults, as called at
                        GPR:73 -- astropy is NOT installed here and the reference
                        pins no version: restated from astropy's documented
                        algorithm (kernel: Gaussian2D model sampled at pixel
                        centres, size = 8*std rounded up to odd, normalised to
                        unit sum; convolve: boundary='fill' with 0,
                        nan_treatment='interpolate' = per-pixel renormalisation
                        over the non-NaN window entries, NaN where the whole
                        window is NaN).  **parity unpinned** against astropy.
* ``smooth``         <- GPR:65-76
* ``numpy_pairwise_sum`` -- numpy's summation order (8192-element iterator
                        buffers, each pairwise: PW_BLOCKSIZE 128, 8
                        accumulators), which ``np.nanmean``
                        uses at GPR:74; the HIP smoothing kernel reproduces it so
                        smoothing is bit-exact against this oracle
                        (``tests/test_day_oracle.py`` pins it to ``np.sum``).
* ``interpolate_day`` <- GPR:200-336 for one rank (pass 1 GPR3D(opt=True) per
                        cell, smooth the 5 hyper fields GPR:299-307, pass 2
                        GPR3D(opt=False) GPR:314-330), returning the same dict keys.
"""
import numpy as np

from . import gp_oracle as G


# ------------------------------------------------------------ GPR:223-246
def training_set(sat, x, y):
    """sat (nx, ny, 4, T) binned freeboard (NaN = no obs), x/y (nx, ny) grid
    coordinates -> x_train, y_train, t_train, z in the reference's order:
    satellite-major, then day, then np.where order of the grid."""
    nsat, T = sat.shape[2], sat.shape[3]
    xs = [[] for _ in range(nsat)]
    ys = [[] for _ in range(nsat)]
    ts = [[] for _ in range(nsat)]
    zs = [[] for _ in range(nsat)]
    for day in range(T):
        for s in range(nsat):
            ids = np.where(~np.isnan(sat[:, :, s, day]))
            xs[s].extend(x[ids])
            ys[s].extend(y[ids])
            ts[s].extend(np.ones(np.shape(ids)[1]) * day)
            zs[s].extend(sat[:, :, s, day][ids])
    return (np.concatenate(xs), np.concatenate(ys), np.concatenate(ts), np.concatenate(zs))


# ------------------------------------------------------------ GPR:159
def ball_query(pts, q, r):
    """Indices of the rows of ``pts`` (M x 2) within distance r of ``q`` (2,),
    ascending.  Distance test as scipy's cKDTree for p=2:
    (dx*dx + dy*dy) <= r*r, dims accumulated in order."""
    dx = pts[:, 0] - q[0]
    dy = pts[:, 1] - q[1]
    d2 = dx * dx
    d2 = d2 + dy * dy
    return np.nonzero(d2 <= r * r)[0]


# ------------------------------------------------------------ astropy, GPR:73
def _round_up_to_odd_integer(value):
    i = int(np.ceil(value))
    return i + 1 if i % 2 == 0 else i


def gaussian2d_kernel(std):
    """astropy.convolution.Gaussian2DKernel(x_stddev=std, y_stddev=std): the
    Gaussian2D model (amplitude 1/(2 pi sx sy), theta 0) evaluated at integer
    offsets (discretize mode 'center'), then normalised to unit sum."""
    size = _round_up_to_odd_integer(8 * std)
    half = (size - 1) // 2
    xr = np.arange(-half, half + 1)
    xx, yy = np.meshgrid(xr, xr)
    theta = 0.0
    cost2 = np.cos(theta) ** 2
    sint2 = np.sin(theta) ** 2
    sin2t = np.sin(2. * theta)
    xstd2 = std ** 2
    ystd2 = std ** 2
    a = 0.5 * ((cost2 / xstd2) + (sint2 / ystd2))
    b = 0.5 * ((sin2t / xstd2) - (sin2t / ystd2))
    c = 0.5 * ((sint2 / xstd2) + (cost2 / ystd2))
    amp = 1. / (2 * np.pi * std * std)
    arr = amp * np.exp(-((a * xx ** 2) + (b * xx * yy) + (c * yy ** 2)))
    return arr / arr.sum()


def convolve_interpolate(data, kern, fill_value=0.0):
    """astropy.convolution.convolve(data, kern) with its defaults
    (boundary='fill', fill_value=0, nan_treatment='interpolate',
    normalize_kernel=True, preserve_nan=False): for every pixel
    top = sum val*ker, bot = sum ker over the non-NaN entries of the window
    (rows outer, columns inner, kernel flipped; padding counts as a valid 0),
    result = top / bot, NaN when bot == 0."""
    ny, nx = data.shape
    ky, kx = kern.shape
    wy, wx = ky // 2, kx // 2
    pad = np.full((ny + 2 * wy, nx + 2 * wx), fill_value, dtype=np.float64)
    pad[wy:wy + ny, wx:wx + nx] = data
    top = np.zeros((ny, nx))
    bot = np.zeros((ny, nx))
    for ii in range(ky):
        for jj in range(kx):
            ker = kern[ky - 1 - ii, kx - 1 - jj]
            val = pad[ii:ii + ny, jj:jj + nx]
            ok = ~np.isnan(val)
            top = np.where(ok, top + val * ker, top)
            bot = np.where(ok, bot + ker, bot)
    with np.errstate(invalid='ignore', divide='ignore'):
        res = np.where(bot == 0, np.nan, top / np.where(bot == 0, 1.0, bot))
    return res


def smooth(data, vmax, mask, std=1):
    """GPR:65-76."""
    data_smth = np.copy(data)
    data_smth[np.isinf(data_smth)] = np.nan
    with np.errstate(invalid='ignore'):
        data_smth[data_smth > vmax] = vmax
    data_smth = convolve_interpolate(data_smth, gaussian2d_kernel(std))
    data_smth[data_smth == 0] = np.nanmean(data_smth)
    data_smth[np.isnan(mask)] = np.nan
    return data_smth


def numpy_pairwise_sum(a, block=8192):
    """np.sum of a contiguous float64 array, in numpy's order: the reduction
    runs over iterator buffers of 8192 elements, each summed pairwise
    (blocks <= 128 with 8 accumulators, halves rounded to multiples of 8),
    the block sums accumulated left to right onto 0.0."""
    a = np.asarray(a, dtype=np.float64).reshape(-1)

    def pw(lo, n):
        if n < 8:
            res = 0.
            for i in range(n):
                res += a[lo + i]
            return res
        if n <= 128:
            r = [a[lo + k] for k in range(8)]
            i = 8
            while i < n - (n % 8):
                for k in range(8):
                    r[k] += a[lo + i + k]
                i += 8
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
            while i < n:
                res += a[lo + i]
                i += 1
            return res
        n2 = n // 2
        n2 -= n2 % 8
        return pw(lo, n2) + pw(lo + n2, n - n2)

    total = 0.0
    for lo in range(0, len(a), block):
        total += pw(lo, min(block, len(a) - lo))
    return total


SMOOTH_VMAX_KEYS = ('ell_x', 'ell_y', 'ell_t', 'sf2', 'sn2')


def smooth_vmax(radius_km, T):
    """GPR:303-307 clip values for (ell_x, ell_y, ell_t, sf2, sn2)."""
    return (2 * radius_km * 1000, 2 * radius_km * 1000, T, 0.1, 0.05)


# ------------------------------------------------------------ GPR:200-336
def interpolate_day(sat, sie, x, y, mean, date='d', T=9, radius=300, grid_res=25, x0=None,
                    pass1_rows=None):
    """Single-rank restatement of GPR:216-336.  ``sat`` (nx, ny, 4, T) (the
    ``obs[..., day:day+T]`` slice), ``sie`` (nx, ny) with NaN outside the ice.
    ``pass1_rows`` (ncell x 8 GPR3D tuples) replaces pass 1 (tests use it to
    check smoothing + pass 2 independently of the optimiser's trajectory)."""
    from scipy.spatial import cKDTree
    T_mid = T // 2
    x0 = G.X0_PRODUCTION if x0 is None else x0
    x_train, y_train, t_train, z = training_set(sat, x, y)
    IDs = np.where(~np.isnan(sie))
    X = np.array([x[IDs], y[IDs]]).T
    tree = cKDTree(np.array([x_train, y_train]).T)
    res = {}
    fields = {k: np.zeros(sie.shape) * np.nan for k in
              ('interp', 'interp_error', 'lZ', 'ell_x', 'ell_y', 'ell_t', 'sf2', 'sn2')}
    if pass1_rows is None:
        rows = []
        for index in range(X.shape[0]):
            ID = tree.query_ball_point(x=X[index, :], r=radius * 1000)
            inputs = np.array([x_train[ID], y_train[ID], t_train[ID]]).T
            outputs = z[ID]
            rows.append(G.gp_cell(inputs, outputs, np.array([X[index, 0], X[index, 1], T_mid]),
                                  mean, opt=True, x0=x0))
        rows = np.array(rows, dtype=np.float64).reshape(-1, 8)
    else:
        rows = np.asarray(pass1_rows, dtype=np.float64).reshape(-1, 8)
    for k, key in enumerate(('interp', 'interp_error', 'lZ', 'ell_x', 'ell_y', 'ell_t', 'sf2', 'sn2')):
        fields[key][IDs] = rows[:, k]
        res[date + '_' + key] = fields[key]
    std = 2 if grid_res == 25 else 1
    for key, vmax in zip(SMOOTH_VMAX_KEYS, smooth_vmax(radius, T)):
        res[date + '_' + key + '_smth'] = smooth(res[date + '_' + key], vmax, sie, std)
    ellXs = np.array([res[date + '_ell_x_smth'][IDs], res[date + '_ell_y_smth'][IDs],
                      res[date + '_ell_t_smth'][IDs]]).T
    sn2xs = res[date + '_sn2_smth'][IDs]
    sf2xs = res[date + '_sf2_smth'][IDs]
    fs_smth = np.zeros(sie.shape) * np.nan
    sfs2_smth = np.zeros(sie.shape) * np.nan
    out2 = []
    for index in range(X.shape[0]):
        ID = tree.query_ball_point(x=X[index, :], r=radius * 1000)
        inputs = np.array([x_train[ID], y_train[ID], t_train[ID]]).T
        outputs = z[ID]
        hyp = (ellXs[index, 0], ellXs[index, 1], ellXs[index, 2], sf2xs[index], sn2xs[index])
        out2.append(G.gp_cell(inputs, outputs, np.array([X[index, 0], X[index, 1], T_mid]), mean,
                              opt=False, hyp=hyp)[:2])
    out2 = np.array(out2, dtype=np.float64).reshape(-1, 2)
    fs_smth[IDs] = out2[:, 0]
    sfs2_smth[IDs] = out2[:, 1]
    res[date + '_interp_smth'] = fs_smth
    res[date + '_interp_error_smth'] = sfs2_smth
    return res
