"""Stage split of the diagonal factor (diag_tile, csrc/oi_kernels.hip) from
the OI_DIAG_TIMING build (scripts/build_exp_lib.sh diagtime -DOI_DIAG_TIMING):
summed clock64 stamps of every diagonal factor workgroup 0 runs.  GPU only:
    OI_LIB=build_exp/liboi_diagtime.so python3 tools/diag_stage_probe.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (same HIP runtime as liboi)
from optimalinterpolation_amd import _lib, synthetic  # noqa: E402

lib = _lib.load()
f = lib.oi_diag_stamps
f.argtypes = [ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
buf = (ctypes.c_longlong * 16)()
NAMES = ['load/generate', 'potrf', 'L store + logdet', 'trtri diagonal blocks', 'trtri off-diagonal',
         'Dinv store + fwd subst', 'W store + alpha']
X0 = [np.log(25e3), np.log(25e3), np.log(1.0), np.log(1.0), np.log(1.0), np.log(.1)]


def split(label, sizes, seed):
    cells = synthetic.make_cells(sizes, seed=seed)
    _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True)
    f(buf, 1)
    _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True)
    assert f(buf, 0) == 0
    s = np.array(buf[:16], dtype=np.int64)
    calls = int(s[15])
    d = np.diff(s[:8].astype(np.float64)) / max(calls, 1)
    tot = d.sum()
    print(f"{label}: {calls} diagonal factors by workgroup 0, {tot:.0f} cycles each: " +
          ", ".join(f"{n} {v:.0f} ({v / tot:.0%})" for n, v in zip(NAMES, d)), flush=True)


split("config 1 (one n = 200 cell)", [200], 5)
split("64 cells n = 1600", [1600] * 64, 6)
