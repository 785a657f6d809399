"""Per-launch timing of one SMLII round (profile=True), with executed MFMA
TF/s of the panel launches: day-shard mix (1250 cells, n ~ U{300..3000}) and
a homogeneous batch (256 cells, n = 3000)."""
import sys
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic

TP = 2 * 64 ** 3


def run(cells, label):
    nc = cells.ncell
    h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
    mX = np.full(len(cells.z), cells.mean)
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
    _lib.profile_reset()
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True)
    pj = _lib.profile_json()
    Ts = (np.diff(cells.offs) + 63) // 64
    print(f"== {label}: cells={nc} Tmax={Ts.max()}", flush=True)
    tot = {}
    for k, j, c, ms in pj['last_round']:
        tot[k] = tot.get(k, 0.0) + ms
        if k in ('k_chol_panel', 'k_diag_factor', 'k_scale') and j % 4 == 0 or k in ('k_build', 'k_lauum_grad', 'k_zvec', 'k_avec', 'k_finalize'):
            extra = ''
            if k == 'k_chol_panel':
                act = Ts[Ts > j]
                tp = np.sum((act - 1 - j) * (j + 1) + j * (j + 1) / 2 + np.where(act - 1 - j > 0, j + 1, 0))
                extra = f"  {tp * TP / ms / 1e9:6.1f} TF/s executed"
            if k == 'k_lauum_grad':
                tp = sum(np.sum((T - np.arange(T)) * (np.arange(T) + 1)) for T in Ts)
                extra = f"  {tp * TP / ms / 1e9:6.1f} TF/s executed"
            print(f"  {k:14s} j={j:3d} cells={c:5d} {ms:8.3f} ms{extra}")
    print('  totals ms:', {k: round(v, 2) for k, v in tot.items()}, 'sum', round(sum(tot.values()), 2))


day = synthetic.make_day(seed=0)
perm = np.random.default_rng(99).permutation(day.ncell)
run(day.subset(np.sort(perm[0::8])), 'day shard')
run(synthetic.make_cells([3000] * 256, seed=3), 'n=3000 x 256')
run(synthetic.make_cells([1600] * 800, seed=3), 'n=1600 x 800')
