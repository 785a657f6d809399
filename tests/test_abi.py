"""The C-ABI library (include/oi.h) loads and exports every declared symbol.
CPU only: no compute entry point is called here."""
import ctypes
import os
import re
import subprocess

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
