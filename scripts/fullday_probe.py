"""Time one oi_gpr_batch call over the whole synthetic day (9997 cells) on one GPU."""
import sys, time
sys.path.insert(0, '.')
import numpy as np
import torch
from optimalinterpolation_amd import _lib, synthetic
day = synthetic.make_day(seed=0)
x0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])
dev = torch.device('cuda', 0)
small = synthetic.make_cells([300] * 8, seed=1)
_lib.gpr_batch(small.xyt, small.z, small.offs, small.xs, small.mean, x0=x0, opt=True)  # prime
xyt = torch.from_numpy(day.xyt).to(dev)
z = torch.from_numpy(day.z).to(dev)
torch.cuda.synchronize()
for maxpool in [int(a) for a in sys.argv[1:]] or [0]:
    t = time.perf_counter()
    out, st, info = _lib.gpr_batch_device(xyt, z, day.offs, day.xs, day.mean, x0=x0, opt=True, info=True,
                                          device=0, max_pool=maxpool)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"max_pool={maxpool}: {day.ncell} cells in {dt:.1f} s = {day.ncell / dt:.2f} cells/s, evals/cell {info[:, 3].mean():.2f}", flush=True)
