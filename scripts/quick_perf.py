import time, json, sys
import numpy as np
sys.path.insert(0, '.')
from optimalinterpolation_amd import _lib, synthetic
# config 2: 1000 cells n=500 predict-only
cells = synthetic.make_cells([500]*1000, seed=2)
hyp = np.tile(synthetic.FIXED_HYPERS, (1000, 1))
_lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp)
for rep in range(3):
    t=time.time(); _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, opt=False, hyp=hyp); dt=time.time()-t
    print(f"config2 predict 1000x500: {dt*1e3:.2f} ms  -> {1000/dt:.0f} cells/s", flush=True)
# one SMLII eval over a batch of cells of various n
for n, nc in [(500, 1000), (1600, 512), (3000, 256)]:
    cells = synthetic.make_cells([n]*nc, seed=3)
    h = np.tile(np.array([np.log(3e5), np.log(3e5), np.log(10.), np.log(5e-3), np.log(1e-3), 0.]), (nc, 1))
    mX = np.full(len(cells.z), cells.mean)
    _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h)
    _lib.profile_reset()
    t=time.time(); _lib.nlml_grad_batch(cells.xyt, cells.z, mX, cells.offs, h, profile=True); dt=time.time()-t
    pj=_lib.profile_json()
    T=(n+63)//64; fl=nc*(n**3+40*n**2)
    print(f"SMLII batch {nc}x{n}: {dt*1e3:.1f} ms wall, useful {fl/dt/1e12:.2f} TFLOP/s", flush=True)
    for k,v in pj['kernels'].items():
        if v['launches']: print(f"   {k:14s} launches {v['launches']:4d} {v['total_ms']:9.3f} ms  exec {v['flops']/max(v['total_ms'],1e-9)/1e9:7.2f} TF/s")
