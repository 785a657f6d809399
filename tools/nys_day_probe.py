"""Nystrom predict over day-like ragged cells (NB1 GPR(approx=True), default
M = int(n/5)): padded batched factorisations vs per-M batches (diagnostic)."""
import os, sys, time, json
sys.path.insert(0, '/root/repo')
import numpy as np
from optimalinterpolation_amd import _lib, nystrom, synthetic

ncell = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
day = synthetic.make_day(seed=0, max_cells=ncell)
sizes = np.diff(day.offs)
M = np.array([int(n / 5) for n in sizes])
hyp = np.tile(synthetic.FIXED_HYPERS, (day.ncell, 1))
sel, soffs = nystrom._ragged_sel(day.offs, M)
y = day.z - day.mean
out = {}
for pad in ('32', '0'):
    os.environ['OI_NYS_PAD'] = pad
    w = day.offs[8]  # warm-up call on the first 8 cells
    _lib.nystrom_batch(day.xyt[:w], y[:w], day.offs[:9], sel[:soffs[8]], soffs[:9], hyp[:8],
                       xs=day.xs[:8], mean=day.mean, objective=False)
    t = time.time()
    _, _, pred, st = _lib.nystrom_batch(day.xyt, y, day.offs, sel, soffs, hyp, xs=day.xs, mean=day.mean,
                                        objective=False)
    dt = time.time() - t
    out[pad] = (dt, pred)
    print(f"pad quantum {pad}: {day.ncell} cells (n {sizes.min()}..{sizes.max()}, M = n/5) predict in "
          f"{dt:.2f} s = {day.ncell / dt:.0f} cells/s, status {int(st.sum())}", flush=True)
d = np.abs(out['32'][1] - out['0'][1]) / np.maximum(1e-12, np.abs(out['0'][1]))
print("max rel diff padded vs unpadded (fs, sd, prior):", np.nanmax(d, 0))
json.dump({"ncell": int(day.ncell), "padded_s": out['32'][0], "unpadded_s": out['0'][0]},
          open('gpurun_out/nys_day_probe.json', 'w'))
