"""Multi-GPU sharding of a day's cells.

The reference distributes cells round-robin over MPI ranks
(``split``, GPR_CS2S3.py:18-23; ``COMM.scatter`` :256) and gathers the
per-cell tuples back to rank 0 (``COMM.gather`` :262).  Here: one process per
GPU; cells are partitioned by longest-processing-time-first on an n^3 cost
estimate (or the reference's strided split); every rank runs its cells through
one batched liboi call; the ncell x 8 fp64 results come back to rank 0 in one
collective (RCCL over xGMI on GPUs, gloo in CPU tests).  There is no other
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


def cell_costs(sizes, opt=True):
    """Relative cost model: opt cells ~ E(n) * n^3 with E(n) ~ 85 + 0.045 (n - 300)
    (SURVEY.md §6 fit); predict-only cells ~ n^3 / 3."""
    n = np.asarray(sizes, dtype=np.float64)
    if not opt:
        return n ** 3 / 3 + 1.0
    return (85.0 + 0.045 * np.maximum(n - 300.0, 0.0)) * (n ** 3 + 40 * n ** 2) + 1.0


def gather_rows(local_rows, local_idx, ncell, device=None, group=None):
    """Gather per-cell result rows from every rank to rank 0 (one all_gather of
    sizes + one all_gather of the padded [idx | rows] payload).  Returns the
    full (ncell x m) array on rank 0 (rows in global cell order), None elsewhere."""
    import torch
    import torch.distributed as dist
    local_rows = np.asarray(local_rows, dtype=np.float64)
    m = local_rows.shape[1] if local_rows.ndim == 2 else 0
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    k = torch.tensor([len(local_idx)], dtype=torch.int64, device=device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    kmax = int(max(int(x.item()) for x in ks))
    if kmax == 0:  # every rank empty: nothing to exchange
        return np.full((ncell, m), np.nan) if rank == 0 else None
    pay = torch.zeros((kmax, m + 1), dtype=torch.float64, device=device)
    if len(local_idx):
        pay[:len(local_idx), 0] = torch.from_numpy(np.asarray(local_idx, dtype=np.float64))
        pay[:len(local_idx), 1:] = torch.from_numpy(local_rows)
    bufs = [torch.zeros_like(pay) for _ in range(world)]
    dist.all_gather(bufs, pay, group=group)
    if rank != 0:
        return None
    full = np.full((ncell, m), np.nan)
    for r in range(world):
        kr = int(ks[r].item())
        b = bufs[r][:kr].cpu().numpy()
        full[b[:, 0].astype(np.int64)] = b[:, 1:]
    return full


def run_sharded(cells, compute, rank, world, device=None, partition='lpt', opt=True, group=None):
    """Pass 1 over a day on ``world`` ranks.

    ``cells``   synthetic.RaggedCells-like (all ranks hold the same metadata)
    ``compute`` callable(subset_cells) -> (out [k x 8], status [k], info [k x 4])
                (the product passes the liboi batched call; CPU tests pass a stub)
    Returns (full ncell x 13 array on rank 0: out | status | info, else None).
    """
    sizes = cells.sizes
    if partition == 'lpt':
        parts = lpt_partition(cell_costs(sizes, opt), world)
    else:
        parts = strided_partition(cells.ncell, world)
    mine = parts[rank]
    if len(mine):
        out, status, info = compute(cells.subset(mine))
        info = np.zeros((len(mine), 4)) if info is None else info
        rows = np.column_stack([out, status.astype(np.float64), info.astype(np.float64)])
    else:
        rows = np.zeros((0, 13))
    return gather_rows(rows, mine, cells.ncell, device=device, group=group)


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
