import sys; sys.path.insert(0,'.')
import numpy as np
from oracle import gp_oracle as O
from optimalinterpolation_amd import _lib, synthetic
def nlz_at(hyp5, x, y, mean):
    h = np.r_[np.log(hyp5), np.log(.1)]
    f, _ = O.neg_log_ml(h, x, y, np.ones(len(y)) * mean)
    return float(np.asarray(f).item()) if np.ndim(f) else float(f)
rng = np.random.default_rng(77)
sizes = rng.integers(20, 260, 40)
cells = synthetic.make_cells(sizes, seed=78)
out, status, info = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=np.array(O.X0_PRODUCTION), opt=True, info=True)
prng = np.random.default_rng(5)
for c in range(cells.ncell):
    x, y, xs = cells.cell(c)
    tr=[]; ref = np.array(O.gp_cell(x, y, xs[0], cells.mean, opt=True, trace=tr), float)
    fg = nlz_at(out[c,3:8], x, y, cells.mean); fr = nlz_at(ref[3:8], x, y, cells.mean)
    perm_f=[]; perm_fs=[]
    for k in range(3):
        p = prng.permutation(len(y))
        rp = np.array(O.gp_cell(x[p], y[p], xs[0], cells.mean, opt=True), float)
        perm_f.append(nlz_at(rp[3:8], x, y, cells.mean)); perm_fs.append(rp[0])
    print(f"c{c:2d} n={len(y):3d} ev {info[c,3]:3d}/{len(tr):3d} cg {info[c,1]} fs_rel {abs(out[c,0]-ref[0])/abs(ref[0]):.1e} "
          f"f_gpu-f_ref {fg-fr:+.2e} perm(f-f_ref) [{min(perm_f)-fr:+.2e},{max(perm_f)-fr:+.2e}] perm_fs_rel {max(abs(np.array(perm_fs)-ref[0]))/abs(ref[0]):.1e}", flush=True)
