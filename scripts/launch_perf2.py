"""Per-launch timing of one SMLII round (profile=True) in the default
paired-column scheme: for every column step j, the times of k_diag_factor,
k_scale, k_panel_even (j even) / k_chol_panel (j odd) and their executed MFMA
TF/s (tile-product counts as in oi_engine.cpp's profile accounting)."""
import sys
sys.path.insert(0, '.')
import numpy as np
from optimalinterpolation_amd import _lib, synthetic

TP = 2 * 64 ** 3


def products(kind, T, j):
    """executed tile products of one launch for one cell of T tiles (eval mode)"""
    if T <= j:
        return 0
    if kind == 'k_panel_even':
        p = 2 * (T - 1 - j) * (j + 1) + (1 if T - 1 - j > 0 else 0)
        return p + sum(2 * (j - jj) for jj in range(j))
    if kind == 'k_chol_panel':
        kbeg = j - 1
        p = (T - 1 - j) * (j + 1 - kbeg) + ((j + 1) if T - 1 - j > 0 else 0)
        return p + sum(j - max(jj, kbeg) + (1 if kbeg > jj else 0) for jj in range(j))
    if kind == 'k_scale':
        return j - (0 if j % 2 == 0 else j - 1)
    return 0


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
        extra = ''
        if k in ('k_panel_even', 'k_chol_panel', 'k_scale'):
            tp = sum(products(k, int(T), j) for T in Ts)
            extra = f"  {tp * TP / ms / 1e9:6.1f} TF/s executed ({tp} products)"
        if k == 'k_lauum_grad':
            tp = sum(np.sum((T - np.arange(T)) * (np.arange(T) + 1)) for T in Ts)
            extra = f"  {tp * TP / ms / 1e9:6.1f} TF/s executed"
        if j < 0 or j % 6 in (0, 1) or j >= Ts.max() - 2:
            print(f"  {k:14s} j={j:3d} cells={c:5d} {ms:8.3f} ms{extra}")
    print('  totals ms:', {k: round(v, 2) for k, v in tot.items()}, 'sum', round(sum(tot.values()), 2), flush=True)


if __name__ == '__main__':
    run(synthetic.make_cells([3000] * 256, seed=3), 'n=3000 x 256')
    run(synthetic.make_cells([1600] * 800, seed=3), 'n=1600 x 800')
