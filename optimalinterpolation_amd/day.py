"""One pan-Arctic day end to end: the reference production script
``2021_paper_production/GPR_CS2S3.py`` (``GPR:``) as a library.

Reference flow (GPR:200-336), one MPI rank per core:
  read pickles (GPR:25-63) -> flatten 4 satellites x T days into a training
  set (GPR:223-246) -> cKDTree (GPR:250) -> pass 1: GPR3D(index) per cell,
  hypers fitted by CG (GPR:258-261) -> gather to rank 0 (GPR:262) -> map to
  grids and smooth the five hyper fields (GPR:264-307) -> bcast (GPR:311) ->
  pass 2: GPR3D(index, opt=False) with the smoothed hypers (GPR:314-319) ->
  gather (GPR:320) -> dict of 2-D fields pickled (GPR:321-336).

Here, one process per GPU: the training set goes to HBM once, the 300 km
neighbour query (``oi_ball_query``) and the per-cell gather
(``oi_gather_rows``) run on the device, pass 1 and pass 2 are one batched
``oi_gpr_batch`` call each over the rank's cells (device-resident inputs),
the five smoothings are one ``oi_smooth_fields`` call, and the only
collectives are one all_gather of the pass-1 rows (every rank then smooths
the same fields itself -- replacing gather + rank-0 smooth + bcast) and one
gather of the pass-2 rows to rank 0 (driver.gather_rows: the partition is
known on every rank, so each exchange is a single collective).

``neighbours='kdtree'`` keeps the reference's exact neighbour order (scipy
cKDTree on the host, rows shipped over PCIe); the default ``'device'``
returns each cell's neighbours in ascending training-set order, which changes
only the summation order inside a cell (results agree to rounding, T1).
"""
import datetime
import os
import pickle

import numpy as np

from . import _lib
from . import driver

# GPR:303-307 keys and clip values; GPR:298-302 kernel width
HYPER_KEYS = ('ell_x', 'ell_y', 'ell_t', 'sf2', 'sn2')
PASS1_KEYS = ('interp', 'interp_error', 'lZ', 'ell_x', 'ell_y', 'ell_t', 'sf2', 'sn2')


def split(container, count):
    """GPR:18-23: divide tasks over ``count`` workers (strided)."""
    return [container[_i::count] for _i in range(count)]


def smooth_std(grid_res):
    """GPR:298-302."""
    return 2 if grid_res == 25 else 1


def smooth_vmax(radius, T):
    """GPR:303-307: clip values of (ell_x, ell_y, ell_t, sf2, sn2)."""
    return (2 * radius * 1000, 2 * radius * 1000, T, 0.1, 0.05)


def gaussian2d_kernel(std):
    """astropy ``Gaussian2DKernel(x_stddev=std, y_stddev=std)`` (used at GPR:73):
    the Gaussian2D model (amplitude 1/(2 pi std^2), theta 0) sampled at
    integer offsets over 8*std rounded up to odd, normalised to unit sum."""
    size = int(np.ceil(8 * std))
    size = size + 1 if size % 2 == 0 else size
    half = (size - 1) // 2
    r = np.arange(-half, half + 1)
    xx, yy = np.meshgrid(r, r)
    a = 0.5 * ((np.cos(0.0) ** 2 / std ** 2) + (np.sin(0.0) ** 2 / std ** 2))
    b = 0.5 * ((np.sin(0.0) / std ** 2) - (np.sin(0.0) / std ** 2))
    c = 0.5 * ((np.sin(0.0) ** 2 / std ** 2) + (np.cos(0.0) ** 2 / std ** 2))
    arr = (1. / (2 * np.pi * std * std)) * np.exp(-((a * xx ** 2) + (b * xx * yy) + (c * yy ** 2)))
    return arr / arr.sum()


def smooth(data, vmax, mask, std=1, **opt_kw):
    """GPR:65-76 on the GPU (one field; see ``smooth_many`` for several)."""
    return _lib.smooth_fields(np.asarray(data, dtype=np.float64)[None], [vmax], mask,
                              gaussian2d_kernel(std), **opt_kw)[0]


def smooth_many(fields, vmaxs, mask, std=1, **opt_kw):
    """The five smoothings of GPR:303-307 in one device call."""
    return _lib.smooth_fields(np.stack([np.asarray(f, dtype=np.float64) for f in fields]), vmaxs,
                              mask, gaussian2d_kernel(std), **opt_kw)


def training_set(sat, x, y):
    """GPR:223-246 vectorised: satellite-major, then day, then the grid in
    ``np.where`` (row-major) order.  Returns x_train, y_train, t_train, z."""
    nx, ny, nsat, T = sat.shape
    xs, ys, ts, zs = [], [], [], []
    for s in range(nsat):
        v = sat[:, :, s, :].transpose(2, 0, 1)  # (T, nx, ny)
        ok = ~np.isnan(v)
        d, i, j = np.nonzero(ok)                # day-major, then np.where order
        xs.append(x[i, j])
        ys.append(y[i, j])
        ts.append(d.astype(np.float64))
        zs.append(v[d, i, j])
    return np.concatenate(xs), np.concatenate(ys), np.concatenate(ts), np.concatenate(zs)


class _SafeUnpickler(pickle.Unpickler):
    """Input pickles are dicts of numpy arrays (read_and_bin.py:52-54): allow
    exactly the classes those need, nothing that executes code."""
    _OK = {('numpy', 'ndarray'), ('numpy', 'dtype'), ('numpy.core.multiarray', '_reconstruct'),
           ('numpy._core.multiarray', '_reconstruct'), ('numpy.core.multiarray', 'scalar'),
           ('numpy._core.multiarray', 'scalar'), ('builtins', 'dict'), ('collections', 'OrderedDict'),
           ('_codecs', 'encode')}  # how protocol 2 stores bytes

    def find_class(self, module, name):
        if (module, name) in self._OK:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name}")


def _load_pickle(path):
    with open(path, 'rb') as f:
        return _SafeUnpickler(f, encoding='latin1').load()


def readFB(datapath, grid_res, season):
    """GPR:25-63: (obs (x, y, 4, t), sie_mask (x, y, t) with <0.15 -> NaN, dates)."""
    names = ('CS2_SAR', 'CS2_SARIN', 'S3A', 'S3B')
    sats = [_load_pickle(os.path.join(datapath, f'{n}_dailyFB_{grid_res}km_{season}_season.pkl'))
            for n in names]
    sie = _load_pickle(os.path.join(datapath, f'SIE_masking_{grid_res}km_{season}_season.pkl'))
    dates = sorted(str(k) for k in sats[0])
    obs, mask, dates_trim = [], [], []
    for key in dates:
        if key in sats[1] and key in sats[2] and key in sats[3]:
            obs.append([sats[0][key], sats[1][key], sats[2][key], sats[3][key]])
            mask.append(sie[key])
            dates_trim.append(key)
    obs = np.array(obs).transpose(2, 3, 1, 0)
    mask = np.array(mask, dtype=np.float64).transpose(1, 2, 0)
    mask[mask < 0.15] = np.nan
    return obs, mask, dates_trim


def save(dic, path):
    """GPR:192-198."""
    with open(path, 'wb') as f:
        pickle.dump(dic, f, protocol=2)


def write_quicklook(path, fs, sd, x=None, y=None, lat=None, lon=None, date='', fmt='netcdf4', created=None):
    """The quick-look product (``QuickLook Data/CS2S3_<date>_25km_quicklook.nc``:
    lat, lon, radar_freeboard, uncertainty on the 320 x 320 grid, fp64).

    ``fmt='netcdf4'`` (default) writes the reference's own netCDF-4 / HDF5
    layout with the from-scratch writer of ``hdf5nc`` (dimensions lat / lon,
    dimension scales, the reference's attributes); lat / lon default to the
    grid coordinates ``x`` / ``y`` when no geographic grid is given.
    ``fmt='netcdf3'`` keeps the classic netCDF-3 file (scipy.io) of round 2."""
    if fmt == 'netcdf4':
        from . import hdf5nc
        lat = np.asarray(lat if lat is not None else (x if x is not None else np.zeros_like(fs)), dtype=np.float64)
        lon = np.asarray(lon if lon is not None else (y if y is not None else np.zeros_like(fs)), dtype=np.float64)
        return hdf5nc.write_quicklook(path, fs, sd, lat, lon, date=date or '00000000', created=created)
    from scipy.io import netcdf_file
    nx, ny = fs.shape
    with netcdf_file(path, 'w') as f:
        f.createDimension('x', nx)
        f.createDimension('y', ny)
        for name, arr in (('lat', lat), ('lon', lon), ('x', x), ('y', y), ('radar_freeboard', fs),
                          ('uncertainty', sd)):
            if arr is None:
                continue
            v = f.createVariable(name, 'f8', ('x', 'y'))
            v[:] = np.asarray(arr, dtype=np.float64)
    return path


class DayResult(dict):
    """The reference's output dict (GPR:290-307, 333-334) plus run info."""
    info = None


def interpolate_day(sat, sie, x, y, mean, date='', T=9, radius=300, grid_res=25, x0=None,
                    neighbours='device', rank=0, world=1, device=0, group=None, partition='lpt',
                    pass1_rows=None, comm_device=None, **opt_kw):
    """GPR:216-336 for one day on ``world`` ranks (this process = ``rank``).

    ``sat`` (nx, ny, 4, T) binned obs, ``sie`` (nx, ny) ice mask of the
    target day (NaN outside), ``x``/``y`` grid coordinates, ``mean`` prior.
    Returns (on rank 0; None elsewhere when world > 1) a dict with the
    reference's keys ``date+'_interp'`` ... ``'_interp_error_smth'``.
    ``pass1_rows`` (ncell x 8) skips the fit (tests of smoothing + pass 2).
    """
    return interpolate_days([(sat, sie, mean, date)], x, y, T=T, radius=radius, grid_res=grid_res,
                            x0=x0, neighbours=neighbours, rank=rank, world=world, device=device,
                            group=group, partition=partition,
                            pass1_rows=None if pass1_rows is None else [pass1_rows],
                            comm_device=comm_device, **opt_kw)[0]


class _Day:
    """Per-day state of interpolate_days on this rank."""


def _prepare_day(sat, sie, mean, date, x, y, T, rad, neighbours, rank, world, dev, device,
                 partition, fixed, opt_kw):
    """Training set (GPR:223-246), ice cells (GPR:248-249), neighbour query
    (GPR:159) and the rank's gathered inputs in HBM, observations already
    minus the day's prior mean (GPR:163)."""
    import torch
    d = _Day()
    d.sie, d.mean, d.date = sie, float(mean), date
    x_train, y_train, t_train, z = training_set(sat, x, y)
    d.n_train = len(z)
    d.IDs = np.where(~np.isnan(sie))
    X = np.array([x[d.IDs], y[d.IDs]]).T
    d.ncell = X.shape[0]
    d.xs_all = np.column_stack([X, np.full(d.ncell, float(T // 2))])
    if neighbours == 'device':
        pts = torch.from_numpy(np.ascontiguousarray(np.column_stack([x_train, y_train]))).to(dev)
        cols = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (x_train, y_train, t_train, z)]
        qall = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
        d.counts = _count_neighbours(pts, qall, rad, device, opt_kw)
    else:
        from scipy.spatial import cKDTree
        tree = cKDTree(np.array([x_train, y_train]).T)
        id_lists = [tree.query_ball_point(x=X[i, :], r=rad) for i in range(d.ncell)]
        d.counts = np.array([len(l) for l in id_lists], dtype=np.int64)
    if partition == 'lpt':
        parts = driver.lpt_partition(driver.cell_costs(d.counts, opt=not fixed), world)
    else:
        parts = [np.asarray(p, dtype=np.int64) for p in split(np.arange(d.ncell), world)]
    d.parts = parts
    d.mine = parts[rank]
    if neighbours == 'device':
        q = qall[torch.from_numpy(d.mine).to(dev)] if len(d.mine) else qall[:0]
        d.offs, idx = _lib.ball_query_device(pts, q.contiguous(), rad, device=device, **opt_kw)
        d.xyt, zz = _lib.gather_rows_device(cols, idx, device=device, **opt_kw)
    else:
        sel = [np.asarray(id_lists[c], dtype=np.int64) for c in d.mine]
        d.offs = np.zeros(len(d.mine) + 1, dtype=np.int64)
        d.offs[1:] = np.cumsum([len(s_) for s_ in sel])
        cat = np.concatenate(sel) if sel else np.zeros(0, np.int64)
        d.xyt = torch.from_numpy(np.ascontiguousarray(
            np.stack([x_train[cat], y_train[cat], t_train[cat]], axis=1).reshape(-1, 3))).to(dev)
        zz = torch.from_numpy(np.ascontiguousarray(z[cat])).to(dev)
    # outputs - mX with mX = mean (GPR:163): the batched call then runs with a
    # zero prior mean and fs = mean + k*.alpha is completed on the host -- the
    # same two roundings as the reference's, so several days (different means)
    # can share one call
    d.r = zz - d.mean
    d.xs = d.xs_all[d.mine]
    return d


def _batched_call(days, opt, x0, hyps, device, opt_kw):
    """One oi_gpr_batch over the rank's cells of every day; returns per-day
    (rows [k x 8], info [k x 4]) with fs completed by the day's mean."""
    import torch
    live = [d for d in days if len(d.mine)]
    out = {id(d): (np.zeros((0, 8)), np.zeros((0, 4))) for d in days}
    if not live:
        return out
    xyt = torch.cat([d.xyt for d in live]).contiguous()
    r = torch.cat([d.r for d in live]).contiguous()
    offs = np.concatenate([[0]] + [np.diff(d.offs) for d in live]).cumsum().astype(np.int64)
    xs = np.concatenate([d.xs for d in live])
    hyp = np.concatenate([hyps[id(d)] for d in live]) if not opt else None
    rows, st, info = _lib.gpr_batch_device(xyt, r, offs, xs, 0.0, x0=x0 if opt else None, opt=opt,
                                           hyp=hyp, info=True, device=device, **opt_kw)
    a = 0
    for d in live:
        k = len(d.mine)
        rr = rows[a:a + k].copy()
        rr[:, 0] = d.mean + rr[:, 0]  # GPR:180 fs = mean + Kxsx^T A
        out[id(d)] = (rr, np.asarray(info[a:a + k], dtype=np.float64))
        a += k
    return out


def interpolate_days(days, x, y, T=9, radius=300, grid_res=25, x0=None, neighbours='device', rank=0,
                     world=1, device=0, group=None, partition='lpt', pass1_rows=None,
                     comm_device=None, **opt_kw):
    """GPR:216-336 for several days at once (``days`` = list of (sat, sie,
    mean, date) as for ``interpolate_day``; the reference script handles one
    ``day`` per run, GPR:211).  Pass 1 of every day is ONE batched call over
    all days' cells on this rank (cells are independent, so per-cell results
    are bitwise those of day-by-day calls), then each day's hyper fields are
    smoothed, then pass 2 is again one call.  Returns a list of per-day dicts
    (rank 0; Nones elsewhere when world > 1)."""
    import torch
    if x0 is None:
        x0 = [np.log(grid_res * 1000), np.log(grid_res * 1000), np.log(1.), np.log(1.), np.log(1.),
              np.log(.1)]
    x0 = np.asarray(x0, dtype=np.float64)
    # ``device``: GPU ordinal (the product); a torch device string such as
    # 'cpu' is accepted only so the multi-rank plumbing can be tested without
    # a GPU (tests substitute the liboi calls)
    dev = torch.device(device) if isinstance(device, str) else torch.device('cuda', device)
    cdev = dev if comm_device is None else comm_device
    rad = radius * 1000
    timing = {}
    t0 = datetime.datetime.now()
    D = [_prepare_day(sat, sie, mean, date, x, y, T, rad, neighbours, rank, world, dev, device,
                      partition, pass1_rows is not None, opt_kw) for sat, sie, mean, date in days]
    if dev.type == 'cuda':
        torch.cuda.synchronize(dev)
    timing['neighbours_s'] = (datetime.datetime.now() - t0).total_seconds()

    # pass 1 (GPR:258-261), all days in one call
    t1 = datetime.datetime.now()
    if pass1_rows is not None:
        p1 = {id(d): (np.asarray(pr, dtype=np.float64).reshape(-1, 8)[d.mine], np.zeros((len(d.mine), 4)))
              for d, pr in zip(D, pass1_rows)}
    else:
        p1 = _batched_call(D, True, x0, None, device, opt_kw)
    timing['pass1_s'] = (datetime.datetime.now() - t1).total_seconds()

    # per day: pass-1 rows to every rank, grids, smoothing (GPR:262-311)
    t2 = datetime.datetime.now()
    results, hyps = [], {}
    for d in D:
        rows1, info1 = p1[id(d)]
        payload = np.column_stack([rows1, info1]) if len(d.mine) else np.zeros((0, 12))
        if world > 1:
            d.full = driver.gather_rows(payload, d.parts, d.ncell, device=cdev, group=group, to_all=True)
        else:
            d.full = np.full((d.ncell, 12), np.nan)
            d.full[d.mine] = payload
        res = DayResult()
        grids = {}
        for k, key in enumerate(PASS1_KEYS):
            g = np.zeros(d.sie.shape) * np.nan
            g[d.IDs] = d.full[:, k]
            grids[key] = g
            res[d.date + '_' + key] = g
        sm = smooth_many([grids[k] for k in HYPER_KEYS], smooth_vmax(radius, T), d.sie,
                         smooth_std(grid_res), device=device)
        for k, key in enumerate(HYPER_KEYS):
            res[d.date + '_' + key + '_smth'] = sm[k]
        # pass-2 hypers looked up at the cell (GPR:170-172)
        hyps[id(d)] = np.column_stack([sm[k][d.IDs] for k in range(5)])[d.mine]
        results.append(res)
    timing['smooth_s'] = (datetime.datetime.now() - t2).total_seconds()

    # pass 2 (GPR:312-319), all days in one call
    t3 = datetime.datetime.now()
    p2 = _batched_call(D, False, x0, hyps, device, opt_kw)
    timing['pass2_s'] = (datetime.datetime.now() - t3).total_seconds()
    out = []
    for d, res in zip(D, results):
        rows2 = p2[id(d)][0][:, :2]
        if world > 1:
            full2 = driver.gather_rows(rows2, d.parts, d.ncell, device=cdev, group=group)
            if rank != 0:
                out.append(None)
                continue
        else:
            full2 = np.full((d.ncell, 2), np.nan)
            full2[d.mine] = rows2
        for k, key in enumerate(('interp_smth', 'interp_error_smth')):
            g = np.zeros(d.sie.shape) * np.nan
            g[d.IDs] = full2[:, k]
            res[d.date + '_' + key] = g
        timing['total_s'] = (datetime.datetime.now() - t0).total_seconds()
        res.info = {'ncell': d.ncell, 'n_train': d.n_train, 'counts': d.counts,
                    'evals': d.full[:, 11], 'timing': dict(timing), 'neighbours': neighbours}
        out.append(res)
    return out


def _count_neighbours(pts, q, rad, device, opt_kw):
    """Neighbour counts of every target (oi_ball_query without the fill)."""
    offs, _ = _lib.ball_query_device(pts, q, rad, device=device, counts_only=True, **opt_kw)
    return np.diff(offs)
