"""The C-ABI library (include/oi.h) loads and exports every declared symbol.
CPU only: no compute entry point is called here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from optimalinterpolation_amd import _lib

HEADER = os.path.join(ROOT, 'include', 'oi.h')


def declared():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(oi_[a-z0-9_]+)\s*\(', src)))


def test_header_matches_binding_list():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    lib = _lib.load()
    for name in declared():
        assert hasattr(lib, name), name
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r'\b[TW] (oi_\w+)', out))
    assert set(declared()) <= exported


def test_version_and_options_defaults():
    lib = _lib.load()
    assert lib.oi_version() == 1
    o = _lib.OiOptions()
    lib.oi_options_default(ctypes.byref(o))
    assert o.device == 0 and o.maxiter == -1 and o.gtol == 1e-5 and o.pool_bytes == 0


def test_log2pi_constant():
    """The kernels hard-code np.log(2*np.pi) (GPR:128)."""
    import numpy as np
    src = open(os.path.join(ROOT, 'optimalinterpolation_amd', 'csrc', 'oi_kernels.hip')).read()
    val = float(re.search(r'#define LOG2PI ([0-9.e+-]+)', src).group(1))
    assert val == np.log(2 * np.pi)


def test_argument_errors_without_gpu():
    """API misuse is rejected with OI_E_ARG (-1) before any device work, so
    these run on a CPU-only host (GPR3D's numerical failures are NOT errors)."""
    import numpy as np
    lib = _lib.load()
    D = ctypes.POINTER(ctypes.c_double)
    I64 = ctypes.POINTER(ctypes.c_int64)
    p = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))
    xyt = np.zeros((3, 3))
    z = np.zeros(3)
    xs = np.zeros((1, 3))
    out = np.zeros((1, 8))
    bad_offs = np.array([1, 3], dtype=np.int64)          # offs[0] must be 0
    rc = lib.oi_gpr_batch(p(xyt, ctypes.c_double), p(z, ctypes.c_double), p(bad_offs, ctypes.c_int64), 1,
                          p(xs, ctypes.c_double), 0.0, None, 0, None, p(out, ctypes.c_double), None, None,
                          None)
    assert rc == -1 and b'offs' in lib.oi_last_error()
    offs = np.array([0, 3], dtype=np.int64)
    rc = lib.oi_gpr_batch(p(xyt, ctypes.c_double), p(z, ctypes.c_double), p(offs, ctypes.c_int64), 1,
                          p(xs, ctypes.c_double), 0.0, None, 1, None, p(out, ctypes.c_double), None, None,
                          None)                               # opt=1 without x0
    assert rc == -1 and b'x0' in lib.oi_last_error()
    o = np.zeros(2, dtype=np.int64)
    rc = lib.oi_ball_query(None, -1, p(xs[:, :2].copy(), ctypes.c_double), 1, 1.0, p(o, ctypes.c_int64),
                           None, 0, None)
    assert rc == -1
    f = np.zeros((1, 4, 4))
    m = np.zeros((4, 4))
    k = np.ones((4, 4))
    rc = lib.oi_smooth_fields(p(f, ctypes.c_double), 1, 4, 4, p(np.ones(1), ctypes.c_double),
                              p(m, ctypes.c_double), 0.0, p(k, ctypes.c_double), 4,
                              p(f.copy(), ctypes.c_double), None)   # even kernel size
    assert rc == -1 and b'odd' in lib.oi_last_error()
    assert lib.oi_gpr_batch(None, None, p(np.zeros(1, np.int64), ctypes.c_int64), 0, None, 0.0, None, 1,
                            None, None, None, None, None) == 0   # empty batch is a no-op


def test_nystrom_argument_errors():
    """oi_nystrom_batch rejects bad ragged batches before any device work."""
    x = np.zeros((4, 3))
    y = np.zeros(4)
    with pytest.raises(_lib.OiError, match='M <= n'):
        _lib.nystrom_batch(x, y, [0, 4], np.arange(5), [0, 5], np.ones((1, 5)), predict=False)
    with pytest.raises(_lib.OiError, match='inducing index'):
        _lib.nystrom_batch(x, y, [0, 4], np.array([0, 4]), [0, 2], np.ones((1, 5)), predict=False)
    with pytest.raises(_lib.OiError, match='hypers'):
        _lib.nystrom_batch(x, y, [0, 4], np.array([0, 1]), [0, 2], np.zeros((1, 5)), predict=False)


def test_svgp_argument_errors():
    """oi_svgp_batch rejects bad shapes / hypers before any device work."""
    x = np.zeros((4, 3))
    y = np.zeros(4)
    Z = np.zeros((1, 2, 3))
    ok = [[1.0, 1.0, 1.0, 1.0, 0.1, 0.0]]
    with pytest.raises(_lib.OiError, match='M must be'):
        _lib.svgp_batch(x, y, [0, 4], np.zeros((1, 65, 3)), ok, [[0, 0, 0]])
    with pytest.raises(_lib.OiError, match='batch must be'):
        _lib.svgp_batch(x, y, [0, 4], Z, ok, [[0, 0, 0]], batch=300)
    with pytest.raises(_lib.OiError, match='lengthscales'):
        _lib.svgp_batch(x, y, [0, 4], Z, [[1.0, 0.0, 1.0, 1.0, 0.1, 0.0]], [[0, 0, 0]])
    with pytest.raises(_lib.OiError, match='n >= 1'):
        _lib.svgp_batch(x, y, [0, 0, 4], np.zeros((2, 2, 3)), ok * 2, [[0, 0, 0]] * 2)
