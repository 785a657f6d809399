"""Synthetic 25 km pan-Arctic workloads.

The reference reads binned CryoSat-2 / Sentinel-3 freeboard pickles that are
not shipped with it (GPR_CS2S3.py:203-214), so every benchmark and test here
runs on seeded synthetic cells of the same shape:

* grid: 25 km over [0, 8e6]^2 m (read_and_bin.py:32), cell centres are grid
  nodes inside a disc about (4e6, 4e6);
* per cell: n observations at radius 300 km * sqrt(U), angle 2*pi*U around
  the centre, snapped to the 25 km grid (this creates duplicated sites, as
  real multi-satellite data does), day t ~ U{0..8} (T = 9, GPR:206);
* z = 0.25 + 0.05 sin(x/2e5) cos(y/3e5) + 0.01 t + N(0, 0.02^2) [m];
* prior mean 0.28, target xs = (cx, cy, T_mid = 4) (GPR:207, GPR:164).
"""
import numpy as np

GRID_M = 25e3
RADIUS_M = 300e3
T_DAYS = 9
T_MID = T_DAYS // 2
PRIOR_MEAN = 0.28
# SURVEY §8d config 2 fixed hyper-parameters (lx, ly, lt, sf2, sn2)
FIXED_HYPERS = (3e5, 3e5, 10.0, 5e-3, 1e-3)


def cell_obs(rng, cx, cy, n, r_max=RADIUS_M, grid_m=GRID_M):
    """n synthetic observations around (cx, cy): returns (xyt n x 3, z n)."""
    r = r_max * np.sqrt(rng.random(n))
    th = 2 * np.pi * rng.random(n)
    x = np.round((cx + r * np.cos(th)) / grid_m) * grid_m
    y = np.round((cy + r * np.sin(th)) / grid_m) * grid_m
    t = rng.integers(0, T_DAYS, n).astype(np.float64)
    z = (0.25 + 0.05 * np.sin(x / 2e5) * np.cos(y / 3e5) + 0.01 * t
         + rng.normal(0.0, 0.02, n))
    return np.stack([x, y, t], axis=1), z


def day_centres(radius_m=1410e3, centre=(4e6, 4e6), grid_m=GRID_M):
    """Grid nodes of the 320x320 25 km grid inside a disc (~1e4 for 1410 km)."""
    g = np.arange(0.0, 8e6, grid_m)
    gx, gy = np.meshgrid(g, g, indexing='ij')
    m = (gx - centre[0]) ** 2 + (gy - centre[1]) ** 2 <= radius_m ** 2
    return np.stack([gx[m], gy[m]], axis=1)


class RaggedCells:
    """A ragged batch of cells in the layout the C-ABI takes (include/oi.h).

    ``xyt`` (N x 3, row-major), ``z`` (N), ``offs`` (ncell+1, int64),
    ``xs`` (ncell x 3) targets, ``mean`` scalar prior mean.
    """

    def __init__(self, xyt, z, offs, xs, mean):
        self.xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
        self.z = np.ascontiguousarray(z, dtype=np.float64)
        self.offs = np.ascontiguousarray(offs, dtype=np.int64)
        self.xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1, 3)
        self.mean = float(mean)

    @property
    def ncell(self):
        return len(self.offs) - 1

    @property
    def sizes(self):
        return np.diff(self.offs)

    def cell(self, c):
        a, b = self.offs[c], self.offs[c + 1]
        return self.xyt[a:b], self.z[a:b], self.xs[c:c + 1]

    def subset(self, idx):
        idx = np.asarray(idx, dtype=np.int64)
        parts_x, parts_z, offs = [], [], [0]
        for c in idx:
            x, z, _ = self.cell(c)
            parts_x.append(x)
            parts_z.append(z)
            offs.append(offs[-1] + len(z))
        xyt = np.concatenate(parts_x) if parts_x else np.zeros((0, 3))
        zz = np.concatenate(parts_z) if parts_z else np.zeros(0)
        return RaggedCells(xyt, zz, np.array(offs), self.xs[idx], self.mean)


def make_cells(sizes, seed=0, centres=None, mean=PRIOR_MEAN, grid_m=GRID_M):
    """Independent synthetic cells with the given obs counts (observation
    sites snapped to a ``grid_m`` lattice, as binned satellite data are)."""
    rng = np.random.default_rng(seed)
    sizes = np.asarray(sizes, dtype=np.int64)
    if centres is None:
        cen = day_centres()
        centres = cen[rng.integers(0, len(cen), len(sizes))]
    xs_all, zs_all, offs = [], [], [0]
    for (cx, cy), n in zip(centres, sizes):
        x, z = cell_obs(rng, cx, cy, int(n), grid_m=grid_m)
        xs_all.append(x)
        zs_all.append(z)
        offs.append(offs[-1] + int(n))
    xs = np.column_stack([np.asarray(centres, dtype=np.float64).reshape(-1, 2),
                          np.full(len(sizes), float(T_MID))])
    xyt = np.concatenate(xs_all) if xs_all else np.zeros((0, 3))
    z = np.concatenate(zs_all) if zs_all else np.zeros(0)
    return RaggedCells(xyt, z, np.array(offs), xs, mean)


def make_day(seed=0, n_lo=300, n_hi=3000, radius_m=1410e3, max_cells=None):
    """Config 3: a 25 km day, ~1e4 cells, n ~ U{n_lo..n_hi}."""
    rng = np.random.default_rng(seed)
    cen = day_centres(radius_m)
    if max_cells is not None:
        cen = cen[:max_cells]
    sizes = rng.integers(n_lo, n_hi + 1, len(cen))
    return make_cells(sizes, seed=seed + 1, centres=cen)


GRID_12P5_M = 12.5e3


def season_day_plan(seed=0, n_lo=300, n_hi=5000, radius_m=1410e3):
    """Config 5, one day of the season: the 12.5 km grid (640 x 640 over the
    same [0, 8e6]^2 m domain, GPR_CS2S3.py:201-203 with grid_res = 12.5), ~4e4
    cell centres inside the disc, n ~ U{n_lo..n_hi}.  Returns
    (centres [ncell x 2], sizes [ncell]) -- the observations of a cell are
    drawn by ``season_cells`` only for the cells a rank owns."""
    rng = np.random.default_rng(seed)
    cen = day_centres(radius_m, grid_m=GRID_12P5_M)
    sizes = rng.integers(n_lo, n_hi + 1, len(cen))
    return cen, sizes


def season_cells(centres, sizes, idx, seed=0):
    """The cells ``idx`` of a season day: each cell's observations from its
    own stream (seed, cell index), snapped to the 12.5 km lattice, so a rank
    can draw its share without drawing the whole day."""
    parts = [make_cells([int(sizes[c])], seed=(seed, int(c)), centres=centres[c:c + 1], grid_m=GRID_12P5_M)
             for c in np.asarray(idx, dtype=np.int64)]
    if not parts:
        return make_cells([], seed=seed)
    xyt = np.concatenate([p.xyt for p in parts])
    z = np.concatenate([p.z for p in parts])
    offs = np.concatenate([[0], np.cumsum([len(p.z) for p in parts])])
    xs = np.concatenate([p.xs for p in parts])
    return RaggedCells(xyt, z, offs, xs, parts[0].mean)


class BinnedDay:
    """Inputs of one reference day (GPR_CS2S3.py:200-221), synthetic:
    ``sat`` (nx, ny, 4, T) binned freeboard of CS2 SAR, CS2 SARIN, S3A, S3B
    (NaN = no observation; the slice ``obs[:, :, :, day:day+T]`` GPR:214),
    ``sie`` (nx, ny) ice mask of the target day (NaN = no ice, GPR:213),
    ``x``, ``y`` (nx, ny) grid coordinates [m], ``mean`` the prior (GPR:212)."""

    def __init__(self, sat, sie, x, y, mean, date='20181205'):
        self.sat, self.sie, self.x, self.y, self.mean, self.date = sat, sie, x, y, mean, date


def make_binned_day(seed=0, nx=320, grid_m=GRID_M, ice_radius_m=1410e3, obs_radius_m=1700e3,
                    cover=(0.02, 0.18), T=T_DAYS, nsat=4):
    """A synthetic day on the 25 km polar grid: ice inside a disc of
    ``ice_radius_m`` about the grid centre (~1e4 cells at 1410 km), satellite
    coverage of each (cell, satellite, day) slot with probability varying
    smoothly in ``cover`` (=> ~300-3000 observations within 300 km of a cell,
    SURVEY §8d), freeboard field as ``cell_obs``."""
    rng = np.random.default_rng(seed)
    g = np.arange(nx, dtype=np.float64) * grid_m
    x, y = np.meshgrid(g, g, indexing='ij')
    c = g[nx // 2]
    rr = np.sqrt((x - c) ** 2 + (y - c) ** 2)
    sie = np.where(rr <= ice_radius_m, 0.9, np.nan)
    p = cover[0] + (cover[1] - cover[0]) * 0.5 * (1 + np.sin(x / 7e5) * np.cos(y / 9e5))
    p = np.where(rr <= obs_radius_m, p, 0.0)
    sat = np.full((nx, nx, nsat, T), np.nan)
    for d in range(T):
        for s in range(nsat):
            hit = rng.random((nx, nx)) < p
            zf = (0.25 + 0.05 * np.sin(x / 2e5) * np.cos(y / 3e5) + 0.01 * d
                  + 0.01 * s + rng.normal(0.0, 0.02, (nx, nx)))
            sat[:, :, s, d] = np.where(hit, zf, np.nan)
    return BinnedDay(sat, sie, x, y, PRIOR_MEAN)
