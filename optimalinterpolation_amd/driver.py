"""Multi-GPU sharding of a day's cells.

The reference distributes cells round-robin over MPI ranks
(``split``, GPR_CS2S3.py:18-23; ``COMM.scatter`` :256) and gathers the
per-cell tuples back to rank 0 (``COMM.gather`` :262).  Here: one process per
GPU; cells are partitioned by longest-processing-time-first on an E(n) m^3 cost
estimate (m = distinct sites, the size of the problem actually solved) (or the reference's strided split); every rank runs its cells through
one batched liboi call; the ncell x 8 fp64 results come back to rank 0 in one
collective -- a single ``gather`` (every rank computes the same partition, so
no size exchange is needed), RCCL over xGMI on GPUs, gloo in CPU tests.  There is no other
data-path communication: cells are independent.
"""
import numpy as np


def strided_partition(ncell, world):
    """GPR_CS2S3.py:18-23 ``split``: container[r::count]."""
    return [np.arange(r, ncell, world, dtype=np.int64) for r in range(world)]


def lpt_partition(costs, world):
    """Greedy longest-processing-time-first assignment of cells to ranks."""
    costs = np.asarray(costs, dtype=np.float64)
    order = np.argsort(-costs, kind='stable')
    load = np.zeros(world)
    parts = [[] for _ in range(world)]
    for c in order:
        r = int(np.argmin(load))
        parts[r].append(int(c))
        load[r] += costs[c]
    return [np.array(sorted(p), dtype=np.int64) for p in parts]


def site_counts(cells):
    """Distinct (x, y, t) sites per cell: the size m of the m x m problem the
    library solves for a cell of n observations (oi_device.h "Duplicate
    sites")."""
    v = np.ascontiguousarray(cells.xyt).view(np.dtype((np.void, 24))).ravel()
    return np.array([len(np.unique(v[a:b])) for a, b in zip(cells.offs[:-1], cells.offs[1:])], dtype=np.int64)


def expected_sites(sizes, grid_m=25e3, radius_m=300e3, t_days=9):
    """Expected distinct sites of n observations drawn uniformly over the
    lattice nodes of a radius_m disc x t_days days (the synthetic generator,
    SURVEY §8d): S (1 - exp(-n / S)), S = nodes x days.  Used to balance cells
    whose observations a rank has not drawn yet (config 5)."""
    n = np.asarray(sizes, dtype=np.float64)
    S = np.pi * (radius_m / grid_m) ** 2 * t_days
    return S * -np.expm1(-n / S)


# E(n): SMLII evaluations per opt=True cell, least squares on the build's own
# day run (bench.py --dump: info[:, 3] of the 9997 timed cells on MI355X, round
# 3; tests/golden/day_cells_r03.npz): 90.3 per cell at n ~ 300..600 rising to
# 102.7 at 2700..3000 (SURVEY §6's CPU fit, 85 + 0.045 (n - 300), was made on
# 6 cells and overstates the growth 8x)
EVALS_A, EVALS_B = 86.7, 0.0053


def evals_model(sizes):
    n = np.asarray(sizes, dtype=np.float64)
    return EVALS_A + EVALS_B * n


def cell_costs(sizes, opt=True, sites=None):
    """Relative cost model for partitioning cells.  The work of a cell is done
    on its m distinct sites (``sites``; default: ``sizes``, i.e. m = n):
    opt cells E(n) (m^3 + 40 m^2), the SMLII evaluations times the potrf +
    trtri + lauum work per evaluation (SURVEY §8d F_eval); predict-only cells
    m^3 / 3."""
    n = np.asarray(sizes, dtype=np.float64)
    m = n if sites is None else np.asarray(sites, dtype=np.float64)
    if not opt:
        return m ** 3 / 3 + 16 * m ** 2 + 1.0
    return evals_model(n) * (m ** 3 + 40 * m ** 2) + 1.0


def gather_rows(local_rows, parts, ncell, device=None, group=None, to_all=False):
    """The single collective of a sharded pass (GPR:262 / GPR:320 ``COMM.gather``):
    rank r holds the rows of cells ``parts[r]``; the partition is computed
    identically on every rank, so the sizes are known everywhere and one
    ``gather`` to rank 0 of the [kmax x m] padded rows suffices (``to_all``:
    one ``all_gather``, every rank gets the table -- the pass-1 exchange that
    replaces gather + bcast, GPR:262/311).  Over RCCL the payload stays on
    ``device``.  Returns the (ncell x m) table in global cell order on rank 0
    (every rank with ``to_all``), None elsewhere."""
    import torch
    import torch.distributed as dist
    local_rows = np.asarray(local_rows, dtype=np.float64)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    m = local_rows.shape[1] if local_rows.ndim == 2 else 0
    counts = [len(p) for p in parts]
    if len(parts) != world or counts[rank] != local_rows.shape[0]:
        raise ValueError("partition does not match the process group / local rows")
    kmax = max(counts) if counts else 0
    full = np.full((ncell, m), np.nan)
    if kmax == 0:  # every rank empty (e.g. a day without ice): nothing to exchange
        return full if (to_all or rank == 0) else None
    pay = torch.zeros((kmax, m), dtype=torch.float64, device=device)
    if counts[rank]:
        pay[:counts[rank]] = torch.from_numpy(local_rows).to(pay.device)
    if to_all:
        bufs = [torch.empty_like(pay) for _ in range(world)]
        dist.all_gather(bufs, pay, group=group)
    else:
        bufs = [torch.empty_like(pay) for _ in range(world)] if rank == 0 else None
        dist.gather(pay, bufs, dst=dist.get_global_rank(group, 0) if group is not None else 0,
                    group=group)
        if rank != 0:
            return None
    for r in range(world):
        if counts[r]:
            full[np.asarray(parts[r], dtype=np.int64)] = bufs[r][:counts[r]].cpu().numpy()
    return full


def run_sharded(cells, compute, rank, world, device=None, partition='lpt', opt=True, group=None,
                sites=None):
    """Pass 1 over a day on ``world`` ranks.

    ``cells``   synthetic.RaggedCells-like (all ranks hold the same metadata)
    ``compute`` callable(subset_cells) -> (out [k x 8], status [k], info [k x 4])
                (the product passes the liboi batched call; CPU tests pass a stub)
    ``sites``   distinct sites per cell for the cost model (default: counted)
    Returns (full ncell x 13 array on rank 0: out | status | info, else None).
    """
    sizes = cells.sizes
    if partition == 'lpt':
        if sites is None:
            sites = site_counts(cells)
        parts = lpt_partition(cell_costs(sizes, opt, sites), world)
    else:
        parts = strided_partition(cells.ncell, world)
    mine = parts[rank]
    if len(mine):
        out, status, info = compute(cells.subset(mine))
        info = np.zeros((len(mine), 4)) if info is None else info
        rows = np.column_stack([out, status.astype(np.float64), info.astype(np.float64)])
    else:
        rows = np.zeros((0, 13))
    return gather_rows(rows, parts, cells.ncell, device=device, group=group)


def gpu_compute(opt=True, x0=None, hyp=None, **kw):
    """The product compute step for ``run_sharded``: one liboi batched call."""
    from . import _lib

    def f(sub):
        if opt:
            return _lib.gpr_batch(sub.xyt, sub.z, sub.offs, sub.xs, sub.mean, x0=x0, opt=True,
                                  info=True, **kw)
        return _lib.gpr_batch(sub.xyt, sub.z, sub.offs, sub.xs, sub.mean, opt=False,
                              hyp=hyp(sub) if callable(hyp) else hyp, info=True, **kw)
    return f
