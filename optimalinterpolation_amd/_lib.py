"""ctypes binding of liboi.so (include/oi.h).

The shared library is built in-tree by ``make -C optimalinterpolation_amd``
(or ``__graft_entry__.build()``).  It is the product path: there is no CPU
fallback, and every entry point raises if the library or a GPU is missing.

PyTorch is imported first (when present) so that liboi.so binds to the same
HIP runtime instance that torch already loaded (both carry the soname
libamdhip64.so.7); streams handed over from torch are then valid here.
"""
import ctypes
import os
import threading

import numpy as np

try:  # plumbing only: share torch's HIP runtime if torch is in the process
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# OI_LIB: load a differently-built variant (A/B experiments); default the in-tree build
LIB_PATH = os.environ.get('OI_LIB') or os.path.join(_HERE, 'liboi.so')

_lib = None
_lock = threading.Lock()

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int64_p = ctypes.POINTER(ctypes.c_int64)
c_int32_p = ctypes.POINTER(ctypes.c_int32)

# every symbol include/oi.h declares (tests/test_abi.py checks the export list)
EXPORTS = ('oi_options_default', 'oi_gpr_batch', 'oi_nlml_grad_batch', 'oi_cg_create',
           'oi_cg_step', 'oi_cg_feed', 'oi_cg_result', 'oi_cg_destroy', 'oi_last_error',
           'oi_version', 'oi_profile_json', 'oi_profile_reset', 'oi_smooth_fields',
           'oi_ball_query', 'oi_gather_rows', 'oi_nystrom_batch',
           'oi_nystrom_fit_batch', 'oi_svgp_batch', 'oi_svgp_param_count', 'oi_session_create',
           'oi_session_submit', 'oi_session_set_stream', 'oi_session_wait', 'oi_session_done',
           'oi_session_destroy', 'oi_nystrom_session_create', 'oi_nystrom_session_submit',
           'oi_nystrom_session_wait', 'oi_nystrom_session_destroy')


class OiOptions(ctypes.Structure):
    _fields_ = [('device', ctypes.c_int32), ('maxiter', ctypes.c_int32), ('gtol', ctypes.c_double),
                ('stream', ctypes.c_void_p), ('pool_bytes', ctypes.c_int64),
                ('max_pool', ctypes.c_int32), ('profile', ctypes.c_int32),
                ('device_inputs', ctypes.c_int32)]


class OiError(RuntimeError):
    pass


def load():
    """Load liboi.so (once).  Raises OiError when it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise OiError(f"{LIB_PATH} not built: run `make -C {_HERE}` (or __graft_entry__.build())")
        lib = ctypes.CDLL(LIB_PATH)
        lib.oi_options_default.argtypes = [ctypes.POINTER(OiOptions)]
        lib.oi_options_default.restype = None
        lib.oi_gpr_batch.argtypes = [c_double_p, c_double_p, c_int64_p, ctypes.c_int64, c_double_p,
                                     ctypes.c_double, c_double_p, ctypes.c_int32, c_double_p,
                                     c_double_p, c_int32_p, c_int32_p, ctypes.POINTER(OiOptions)]
        lib.oi_gpr_batch.restype = ctypes.c_int
        lib.oi_nlml_grad_batch.argtypes = [c_double_p, c_double_p, c_double_p, c_int64_p,
                                           ctypes.c_int64, c_double_p, c_double_p, c_double_p,
                                           c_int32_p, ctypes.POINTER(OiOptions)]
        lib.oi_nlml_grad_batch.restype = ctypes.c_int
        lib.oi_cg_create.argtypes = [c_double_p, ctypes.c_double, ctypes.c_int32]
        lib.oi_cg_create.restype = ctypes.c_void_p
        lib.oi_cg_step.argtypes = [ctypes.c_void_p, c_double_p]
        lib.oi_cg_step.restype = ctypes.c_int
        lib.oi_cg_feed.argtypes = [ctypes.c_void_p, ctypes.c_double, c_double_p]
        lib.oi_cg_feed.restype = ctypes.c_int
        lib.oi_cg_result.argtypes = [ctypes.c_void_p, c_double_p, c_double_p, c_int32_p, c_int32_p,
                                     c_int64_p, c_int64_p, c_int64_p]
        lib.oi_cg_result.restype = ctypes.c_int
        lib.oi_cg_destroy.argtypes = [ctypes.c_void_p]
        lib.oi_cg_destroy.restype = None
        lib.oi_last_error.argtypes = []
        lib.oi_last_error.restype = ctypes.c_char_p
        lib.oi_version.argtypes = []
        lib.oi_version.restype = ctypes.c_int32
        lib.oi_profile_json.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        lib.oi_profile_json.restype = ctypes.c_int64
        lib.oi_profile_reset.argtypes = []
        lib.oi_profile_reset.restype = None
        lib.oi_smooth_fields.argtypes = [c_double_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                         c_double_p, c_double_p, ctypes.c_double, c_double_p,
                                         ctypes.c_int32, c_double_p, ctypes.POINTER(OiOptions)]
        lib.oi_smooth_fields.restype = ctypes.c_int
        lib.oi_ball_query.argtypes = [c_double_p, ctypes.c_int64, c_double_p, ctypes.c_int64,
                                      ctypes.c_double, c_int64_p, c_int64_p, ctypes.c_int64,
                                      ctypes.POINTER(OiOptions)]
        lib.oi_ball_query.restype = ctypes.c_int
        lib.oi_gather_rows.argtypes = [c_double_p, c_double_p, c_double_p, c_double_p, ctypes.c_int64,
                                       c_int64_p, ctypes.c_int64, c_double_p, c_double_p,
                                       ctypes.POINTER(OiOptions)]
        lib.oi_gather_rows.restype = ctypes.c_int
        lib.oi_nystrom_batch.argtypes = [c_double_p, c_double_p, c_int64_p, ctypes.c_int64,
                                         c_int64_p, c_int64_p, c_double_p, c_double_p,
                                         ctypes.c_double, c_double_p, c_double_p, c_double_p,
                                         c_int32_p, ctypes.POINTER(OiOptions)]
        lib.oi_nystrom_batch.restype = ctypes.c_int
        lib.oi_nystrom_fit_batch.argtypes = [c_double_p, c_double_p, c_int64_p, ctypes.c_int64,
                                             c_int64_p, c_int64_p, c_double_p, c_double_p,
                                             ctypes.c_double, c_double_p, c_int32_p, c_int32_p,
                                             ctypes.POINTER(OiOptions)]
        lib.oi_nystrom_fit_batch.restype = ctypes.c_int
        lib.oi_svgp_param_count.argtypes = [ctypes.c_int32]
        lib.oi_svgp_param_count.restype = ctypes.c_int32
        lib.oi_svgp_batch.argtypes = [c_double_p, c_double_p, c_int64_p, ctypes.c_int64, c_double_p,
                                      ctypes.c_int32, c_double_p, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_uint64, ctypes.c_double, c_double_p,
                                      c_double_p, c_double_p, c_double_p, c_int32_p,
                                      ctypes.POINTER(OiOptions)]
        lib.oi_svgp_batch.restype = ctypes.c_int
        lib.oi_nystrom_session_create.argtypes = [ctypes.POINTER(OiOptions)]
        lib.oi_nystrom_session_create.restype = ctypes.c_void_p
        lib.oi_nystrom_session_submit.argtypes = [ctypes.c_void_p, c_double_p, c_double_p, c_int64_p,
                                                  ctypes.c_int64, c_int64_p, c_int64_p, c_double_p,
                                                  c_double_p, ctypes.c_double, c_double_p, c_int32_p,
                                                  c_int32_p]
        lib.oi_nystrom_session_submit.restype = ctypes.c_int64
        lib.oi_nystrom_session_wait.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        lib.oi_nystrom_session_wait.restype = ctypes.c_int
        lib.oi_nystrom_session_destroy.argtypes = [ctypes.c_void_p]
        lib.oi_nystrom_session_destroy.restype = None
        lib.oi_session_create.argtypes = [ctypes.POINTER(OiOptions)]
        lib.oi_session_create.restype = ctypes.c_void_p
        lib.oi_session_submit.argtypes = [ctypes.c_void_p, c_double_p, c_double_p, c_int64_p,
                                          ctypes.c_int64, c_double_p, ctypes.c_double, c_double_p,
                                          ctypes.c_int32, c_double_p, c_double_p, c_int32_p, c_int32_p]
        lib.oi_session_submit.restype = ctypes.c_int64
        lib.oi_session_set_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.oi_session_set_stream.restype = ctypes.c_int
        lib.oi_session_wait.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        lib.oi_session_wait.restype = ctypes.c_int
        lib.oi_session_done.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        lib.oi_session_done.restype = ctypes.c_int
        lib.oi_session_destroy.argtypes = [ctypes.c_void_p]
        lib.oi_session_destroy.restype = None
        _lib = lib
        return lib


def _ptr(a, ctype):
    return a.ctypes.data_as(ctypes.POINTER(ctype)) if a is not None else None


def _check(rc):
    if rc != 0:
        raise OiError(f"liboi error {rc}: {load().oi_last_error().decode(errors='replace')}")


def options(device=0, maxiter=-1, gtol=1e-5, stream=None, pool_bytes=0, max_pool=0, profile=False,
            device_inputs=False):
    o = OiOptions()
    load().oi_options_default(ctypes.byref(o))
    o.device = int(device)
    o.maxiter = int(maxiter)
    o.gtol = float(gtol)
    o.stream = stream
    o.pool_bytes = int(pool_bytes)
    o.max_pool = int(max_pool)
    o.profile = 1 if profile else 0
    o.device_inputs = 1 if device_inputs else 0
    return o


def gpr_batch(xyt, z, offs, xs, mean, x0=None, opt=True, hyp=None, info=False, **opt_kw):
    """oi_gpr_batch: returns (out [ncell x 8], status [ncell], info [ncell x 4] or None)."""
    lib = load()
    xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
    z = np.ascontiguousarray(z, dtype=np.float64)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1, 3)
    ncell = len(offs) - 1
    if xs.shape[0] != ncell or offs[0] != 0 or offs[-1] != len(z) or xyt.shape[0] != len(z):
        raise ValueError("inconsistent ragged batch")
    out = np.empty((ncell, 8))
    status = np.zeros(ncell, dtype=np.int32)
    inf = np.zeros((ncell, 4), dtype=np.int32) if info else None
    x0a = np.ascontiguousarray(x0, dtype=np.float64) if x0 is not None else None
    hypa = np.ascontiguousarray(hyp, dtype=np.float64).reshape(-1, 5) if hyp is not None else None
    if opt and (x0a is None or x0a.shape != (6,)):
        raise ValueError("opt=True needs x0 of length 6")
    if not opt and (hypa is None or hypa.shape[0] != ncell):
        raise ValueError("opt=False needs hyp [ncell x 5]")
    o = options(**opt_kw)
    rc = lib.oi_gpr_batch(_ptr(xyt, ctypes.c_double), _ptr(z, ctypes.c_double),
                          _ptr(offs, ctypes.c_int64), ncell, _ptr(xs, ctypes.c_double),
                          float(mean), _ptr(x0a, ctypes.c_double), 1 if opt else 0,
                          _ptr(hypa, ctypes.c_double), _ptr(out, ctypes.c_double),
                          _ptr(status, ctypes.c_int32), _ptr(inf, ctypes.c_int32), ctypes.byref(o))
    _check(rc)
    return out, status, inf


def _check_dev(t, device, dtype='float64', n=None, what='tensor'):
    """A device tensor handed to liboi: right dtype, on cuda:<device>,
    contiguous, ``n`` elements (liboi reads 8 bytes per element)."""
    if str(t.dtype) != f'torch.{dtype}':
        raise ValueError(f"{what} must be torch.{dtype}, got {t.dtype}")
    if t.device.type != 'cuda' or (t.device.index if t.device.index is not None else 0) != int(device):
        raise ValueError(f"{what} must live on cuda:{device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous")
    if n is not None and t.numel() != n:
        raise ValueError(f"{what} has {t.numel()} elements, expected {n}")


def _sync_producers(device):
    """The Nystrom / SVGP entry points run on private non-blocking streams:
    wait here until torch's current stream has produced their device inputs."""
    import torch
    torch.cuda.current_stream(int(device)).synchronize()


def _caller_stream(device):
    """torch's current stream on ``device`` as a hipStream_t (None = the
    legacy NULL stream, which the library then waits for itself)."""
    import torch
    h = torch.cuda.current_stream(device).cuda_stream
    return h or None


def gpr_batch_device(xyt_dev, z_dev, offs, xs, mean, x0=None, opt=True, hyp=None, info=False,
                     **opt_kw):
    """oi_gpr_batch with inputs already resident in HBM: ``xyt_dev`` / ``z_dev``
    are fp64 contiguous torch tensors on cuda:``opt_kw['device']``; the
    metadata stays on the host.  Launches are ordered after torch's current
    stream (include/oi.h, stream ordering)."""
    lib = load()
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1, 3)
    ncell = len(offs) - 1
    N = int(offs[-1])
    dev = int(opt_kw.get('device', 0))
    if xs.shape[0] != ncell or offs[0] != 0:
        raise ValueError("inconsistent ragged batch")
    _check_dev(xyt_dev, dev, n=3 * N, what='xyt')
    _check_dev(z_dev, dev, n=N, what='z')
    out = np.empty((ncell, 8))
    status = np.zeros(ncell, dtype=np.int32)
    inf = np.zeros((ncell, 4), dtype=np.int32) if info else None
    x0a = np.ascontiguousarray(x0, dtype=np.float64) if x0 is not None else None
    hypa = np.ascontiguousarray(hyp, dtype=np.float64).reshape(-1, 5) if hyp is not None else None
    opt_kw.setdefault('stream', _caller_stream(dev))
    o = options(device_inputs=True, **opt_kw)
    rc = lib.oi_gpr_batch(ctypes.cast(xyt_dev.data_ptr(), c_double_p),
                          ctypes.cast(z_dev.data_ptr(), c_double_p),
                          _ptr(offs, ctypes.c_int64), ncell, _ptr(xs, ctypes.c_double),
                          float(mean), _ptr(x0a, ctypes.c_double), 1 if opt else 0,
                          _ptr(hypa, ctypes.c_double), _ptr(out, ctypes.c_double),
                          _ptr(status, ctypes.c_int32), _ptr(inf, ctypes.c_int32), ctypes.byref(o))
    _check(rc)
    return out, status, inf


class Session:
    """oi_session_*: continuous batching across calls (include/oi.h).

    ``submit`` takes the oi_gpr_batch arguments (host numpy arrays, or fp64
    device tensors with ``device_inputs=True``) and returns a ticket;
    ``wait(ticket)`` returns that batch's (out, status, info) once complete,
    leaving later batches' rounds running on the GPU.  Cells of consecutive
    batches share rounds, so a stream of small batches runs at the rate of one
    big call; per-cell results equal oi_gpr_batch's bit for bit.

    Device inputs are ordered after torch's current stream AT EACH SUBMIT
    (oi_session_set_stream), so a producer running under another
    ``torch.cuda.stream(...)`` context is waited for.  Results of a ticket are
    collected once: by ``wait(ticket)``, or in the dict ``wait()`` returns."""

    def __init__(self, device=0, device_inputs=False, **opt_kw):
        self._lib = load()
        self.device = int(device)
        self.device_inputs = bool(device_inputs)
        if self.device_inputs:
            opt_kw.setdefault('stream', _caller_stream(self.device))
        self._opts = options(device=device, device_inputs=device_inputs, **opt_kw)
        self._h = self._lib.oi_session_create(ctypes.byref(self._opts))
        if not self._h:
            raise OiError(f"oi_session_create: {self._lib.oi_last_error().decode(errors='replace')}")
        self._live = {}    # ticket -> results (and the inputs they keep alive), not yet complete
        self._done = {}    # ticket -> results completed by wait(-1), not yet collected

    def submit(self, xyt, z, offs, xs, mean, x0=None, opt=True, hyp=None):
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(-1, 3)
        ncell = len(offs) - 1
        N = int(offs[-1]) if ncell >= 0 else 0
        if xs.shape[0] != ncell or offs[0] != 0:
            raise ValueError("inconsistent ragged batch")
        if self.device_inputs:
            _check_dev(xyt, self.device, n=3 * N, what='xyt')
            _check_dev(z, self.device, n=N, what='z')
            px, pz = _dptr(xyt), _dptr(z)
            _check(self._lib.oi_session_set_stream(self._h, _caller_stream(self.device)))
        else:
            xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
            z = np.ascontiguousarray(z, dtype=np.float64)
            if xyt.shape[0] != N or len(z) != N:
                raise ValueError("inconsistent ragged batch")
            px, pz = _ptr(xyt, ctypes.c_double), _ptr(z, ctypes.c_double)
        x0a = np.ascontiguousarray(x0, dtype=np.float64) if x0 is not None else None
        hypa = np.ascontiguousarray(hyp, dtype=np.float64).reshape(-1, 5) if hyp is not None else None
        if opt and (x0a is None or x0a.shape != (6,)):
            raise ValueError("opt=True needs x0 of length 6")
        if not opt and (hypa is None or hypa.shape[0] != ncell):
            raise ValueError("opt=False needs hyp [ncell x 5]")
        out = np.empty((ncell, 8))
        status = np.zeros(ncell, dtype=np.int32)
        info = np.zeros((ncell, 4), dtype=np.int32)
        t = self._lib.oi_session_submit(self._h, px, pz, _ptr(offs, ctypes.c_int64), ncell,
                                        _ptr(xs, ctypes.c_double), float(mean),
                                        _ptr(x0a, ctypes.c_double), 1 if opt else 0,
                                        _ptr(hypa, ctypes.c_double), _ptr(out, ctypes.c_double),
                                        _ptr(status, ctypes.c_int32), _ptr(info, ctypes.c_int32))
        if t < 0:
            _check(int(t))
        # device inputs and the outputs must outlive the ticket
        self._live[int(t)] = (out, status, info, xyt, z)
        return int(t)

    def done(self, ticket):
        return self._lib.oi_session_done(self._h, int(ticket)) == 1

    def wait(self, ticket=-1):
        """Block until ``ticket`` completes and return its (out, status, info).
        ``ticket = -1`` drains all submitted work and returns
        ``{ticket: (out, status, info)}`` for every ticket not collected yet
        (those can still be collected one by one with ``wait(ticket)``)."""
        ticket = int(ticket)
        if ticket >= 0:
            if ticket in self._done:
                return self._done.pop(ticket)
            if ticket not in self._live:
                raise KeyError(f"unknown or already collected session ticket {ticket}")
        _check(self._lib.oi_session_wait(self._h, ticket))
        if ticket < 0:
            for t, (out, status, info, _, _) in self._live.items():
                self._done[t] = (out, status, info)
            self._live.clear()
            return dict(self._done)
        out, status, info, _, _ = self._live.pop(ticket)
        return out, status, info

    def close(self):
        if getattr(self, '_h', None):
            self._lib.oi_session_destroy(self._h)
            self._h = None
            self._live.clear()
            self._done.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def nlml_grad_batch(xyt, y, mX, offs, h, **opt_kw):
    """oi_nlml_grad_batch: returns (nlz [ncell], grad [ncell x 6], status [ncell])."""
    lib = load()
    xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
    y = np.ascontiguousarray(y, dtype=np.float64)
    mX = np.ascontiguousarray(mX, dtype=np.float64)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    h = np.ascontiguousarray(h, dtype=np.float64).reshape(-1, 6)
    ncell = len(offs) - 1
    if h.shape[0] != ncell or offs[-1] != len(y) or len(mX) != len(y) or xyt.shape[0] != len(y):
        raise ValueError("inconsistent ragged batch")
    nlz = np.empty(ncell)
    grad = np.empty((ncell, 6))
    status = np.zeros(ncell, dtype=np.int32)
    o = options(**opt_kw)
    rc = lib.oi_nlml_grad_batch(_ptr(xyt, ctypes.c_double), _ptr(y, ctypes.c_double),
                                _ptr(mX, ctypes.c_double), _ptr(offs, ctypes.c_int64), ncell,
                                _ptr(h, ctypes.c_double), _ptr(nlz, ctypes.c_double),
                                _ptr(grad, ctypes.c_double), _ptr(status, ctypes.c_int32),
                                ctypes.byref(o))
    _check(rc)
    return nlz, grad, status


def nystrom_batch(xyt, y, offs, sel, soffs, hyp, xs=None, mean=0.0, objective=True,
                  predict=True, **opt_kw):
    """oi_nystrom_batch: returns (nlz [ncell] | None, grad [ncell x 5] | None,
    pred [ncell x 3] | None, status [ncell]).  ``hyp`` are LINEAR hypers
    (ell_x, ell_y, ell_t, sf2, sn2) per cell; ``sel``/``soffs`` the ragged
    inducing rows (0-based within each cell)."""
    lib = load()
    xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
    y = np.ascontiguousarray(y, dtype=np.float64)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    sel = np.ascontiguousarray(sel, dtype=np.int64)
    soffs = np.ascontiguousarray(soffs, dtype=np.int64)
    ncell = len(offs) - 1
    hyp = np.ascontiguousarray(hyp, dtype=np.float64).reshape(ncell, 5)
    if offs[-1] != len(y) or xyt.shape[0] != len(y) or len(soffs) != ncell + 1 \
            or soffs[-1] != len(sel):
        raise ValueError("inconsistent ragged batch")
    if predict:
        xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(ncell, 3)
    nlz = np.empty(ncell) if objective else None
    grad = np.empty((ncell, 5)) if objective else None
    pred = np.empty((ncell, 3)) if predict else None
    status = np.zeros(ncell, dtype=np.int32)
    o = options(**opt_kw)
    rc = lib.oi_nystrom_batch(_ptr(xyt, ctypes.c_double), _ptr(y, ctypes.c_double),
                              _ptr(offs, ctypes.c_int64), ncell, _ptr(sel, ctypes.c_int64),
                              _ptr(soffs, ctypes.c_int64), _ptr(hyp, ctypes.c_double),
                              _ptr(xs if predict else None, ctypes.c_double), float(mean),
                              _ptr(nlz, ctypes.c_double), _ptr(grad, ctypes.c_double),
                              _ptr(pred, ctypes.c_double), _ptr(status, ctypes.c_int32),
                              ctypes.byref(o))
    _check(rc)
    return nlz, grad, pred, status


def nystrom_fit_batch(xyt, y, offs, sel, soffs, x0, xs, mean, **opt_kw):
    """oi_nystrom_fit_batch: returns (out [ncell x 8] = (fs, sd, prior sd, 5 linear
    hypers), status [ncell], info [ncell x 4]).  With device_inputs=True, xyt
    and y are torch device tensors."""
    lib = load()
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    sel = np.ascontiguousarray(sel, dtype=np.int64)
    soffs = np.ascontiguousarray(soffs, dtype=np.int64)
    ncell = len(offs) - 1
    x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(5)
    xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(ncell, 3)
    if opt_kw.get('device_inputs'):
        if xyt.numel() != 3 * offs[-1] or y.numel() != offs[-1]:
            raise ValueError("inconsistent ragged batch")
        px, py = _dptr(xyt), _dptr(y)
        _sync_producers(opt_kw.get('device', 0))
    else:
        xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
        y = np.ascontiguousarray(y, dtype=np.float64)
        if offs[-1] != len(y) or xyt.shape[0] != len(y):
            raise ValueError("inconsistent ragged batch")
        px, py = _ptr(xyt, ctypes.c_double), _ptr(y, ctypes.c_double)
    if len(soffs) != ncell + 1 or soffs[-1] != len(sel):
        raise ValueError("inconsistent inducing rows")
    out = np.empty((ncell, 8))
    status = np.zeros(ncell, dtype=np.int32)
    info = np.zeros((ncell, 4), dtype=np.int32)
    o = options(**opt_kw)
    rc = lib.oi_nystrom_fit_batch(px, py, _ptr(offs, ctypes.c_int64), ncell,
                                  _ptr(sel, ctypes.c_int64), _ptr(soffs, ctypes.c_int64),
                                  _ptr(x0, ctypes.c_double), _ptr(xs, ctypes.c_double), float(mean),
                                  _ptr(out, ctypes.c_double), _ptr(status, ctypes.c_int32),
                                  _ptr(info, ctypes.c_int32), ctypes.byref(o))
    _check(rc)
    return out, status, info


class NystromSession:
    """oi_nystrom_session_*: Nystrom fits (oi_nystrom_fit_batch) as a stream of
    batches with continuous batching across calls.  ``submit`` takes
    nystrom_fit_batch's arguments and returns a ticket; ``wait(ticket)``
    returns that batch's (out, status, info) once its last cell is fitted and
    predicted.  Device inputs (``device_inputs=True``) must stay alive until
    their ticket completes (the session keeps a reference)."""

    def __init__(self, device=0, device_inputs=False, **opt_kw):
        self._lib = load()
        self.device = int(device)
        self.device_inputs = bool(device_inputs)
        self._opts = options(device=device, device_inputs=device_inputs, **opt_kw)
        self._h = self._lib.oi_nystrom_session_create(ctypes.byref(self._opts))
        if not self._h:
            raise OiError(f"oi_nystrom_session_create: {self._lib.oi_last_error().decode(errors='replace')}")
        self._live = {}

    def submit(self, xyt, y, offs, sel, soffs, x0, xs, mean):
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        sel = np.ascontiguousarray(sel, dtype=np.int64)
        soffs = np.ascontiguousarray(soffs, dtype=np.int64)
        ncell = len(offs) - 1
        x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(5)
        xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(ncell, 3)
        if self.device_inputs:
            _check_dev(xyt, self.device, n=3 * int(offs[-1]), what='xyt')
            _check_dev(y, self.device, n=int(offs[-1]), what='y')
            px, py = _dptr(xyt), _dptr(y)
            _sync_producers(self.device)
        else:
            xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
            y = np.ascontiguousarray(y, dtype=np.float64)
            if offs[-1] != len(y) or xyt.shape[0] != len(y):
                raise ValueError("inconsistent ragged batch")
            px, py = _ptr(xyt, ctypes.c_double), _ptr(y, ctypes.c_double)
        if len(soffs) != ncell + 1 or soffs[-1] != len(sel):
            raise ValueError("inconsistent inducing rows")
        out = np.empty((ncell, 8))
        status = np.zeros(ncell, dtype=np.int32)
        info = np.zeros((ncell, 4), dtype=np.int32)
        t = self._lib.oi_nystrom_session_submit(self._h, px, py, _ptr(offs, ctypes.c_int64), ncell,
                                                _ptr(sel, ctypes.c_int64), _ptr(soffs, ctypes.c_int64),
                                                _ptr(x0, ctypes.c_double), _ptr(xs, ctypes.c_double),
                                                float(mean), _ptr(out, ctypes.c_double),
                                                _ptr(status, ctypes.c_int32), _ptr(info, ctypes.c_int32))
        if t < 0:
            _check(int(t))
        self._live[int(t)] = (out, status, info, xyt, y)
        return int(t)

    def wait(self, ticket):
        ticket = int(ticket)
        if ticket not in self._live:
            raise KeyError(f"unknown or already collected session ticket {ticket}")
        _check(self._lib.oi_nystrom_session_wait(self._h, ticket))
        out, status, info, _, _ = self._live.pop(ticket)
        return out, status, info

    def close(self):
        if getattr(self, '_h', None):
            self._lib.oi_nystrom_session_destroy(self._h)
            self._h = None
            self._live.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()


def svgp_batch(xyt, y, offs, Z0, init, xs, batch=100, iterations=10000, log_every=10, seed=0,
               lr=1e-3, want_params=False, **opt_kw):
    """oi_svgp_batch: returns (pred [ncell x 2] = (mean, variance of f), status,
    params [ncell x P] or None, elbo [ncell x nlog] or None).
    Z0 [ncell x M x 3]; init [ncell x 6] = (ls_x, ls_y, ls_t, kernel var, noise var, mean)."""
    lib = load()
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    ncell = len(offs) - 1
    Z0 = np.ascontiguousarray(Z0, dtype=np.float64).reshape(ncell, -1, 3)
    M = Z0.shape[1]
    init = np.ascontiguousarray(init, dtype=np.float64).reshape(ncell, 6)
    xs = np.ascontiguousarray(xs, dtype=np.float64).reshape(ncell, 3)
    if opt_kw.get('device_inputs'):
        if xyt.numel() != 3 * offs[-1] or y.numel() != offs[-1]:
            raise ValueError("inconsistent ragged batch")
        px, py = _dptr(xyt), _dptr(y)
        _sync_producers(opt_kw.get('device', 0))
    else:
        xyt = np.ascontiguousarray(xyt, dtype=np.float64).reshape(-1, 3)
        y = np.ascontiguousarray(y, dtype=np.float64)
        if offs[-1] != len(y) or xyt.shape[0] != len(y):
            raise ValueError("inconsistent ragged batch")
        px, py = _ptr(xyt, ctypes.c_double), _ptr(y, ctypes.c_double)
    P = int(lib.oi_svgp_param_count(M))
    nlog = (iterations + log_every - 1) // log_every if log_every else 0
    pred = np.empty((ncell, 2))
    status = np.zeros(ncell, dtype=np.int32)
    params = np.empty((ncell, P)) if want_params else None
    elbo = np.empty((ncell, nlog)) if nlog else None
    o = options(**opt_kw)
    rc = lib.oi_svgp_batch(px, py, _ptr(offs, ctypes.c_int64), ncell, _ptr(Z0, ctypes.c_double), M,
                           _ptr(init, ctypes.c_double), int(batch), int(iterations), int(log_every),
                           int(seed), float(lr), _ptr(xs, ctypes.c_double), _ptr(pred, ctypes.c_double),
                           _ptr(params, ctypes.c_double), _ptr(elbo, ctypes.c_double),
                           _ptr(status, ctypes.c_int32), ctypes.byref(o))
    _check(rc)
    return pred, status, params, elbo


class CG:
    """The host optimiser (scipy CG restated in C++), driven from Python."""

    def __init__(self, x0, gtol=1e-5, maxiter=-1):
        self._lib = load()
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        self._h = self._lib.oi_cg_create(_ptr(x0, ctypes.c_double), float(gtol), int(maxiter))
        if not self._h:
            raise OiError(self._lib.oi_last_error().decode())
        self._x = np.empty(6)

    def step(self):
        """None when finished, else the point (6,) whose f, g are needed."""
        rc = self._lib.oi_cg_step(self._h, _ptr(self._x, ctypes.c_double))
        if rc < 0:
            _check(rc)
        return None if rc == 0 else self._x.copy()

    def feed(self, f, g):
        g = np.ascontiguousarray(g, dtype=np.float64)
        _check(self._lib.oi_cg_feed(self._h, float(f), _ptr(g, ctypes.c_double)))

    def result(self):
        x = np.empty(6)
        fun = ctypes.c_double()
        nit = ctypes.c_int32()
        st = ctypes.c_int32()
        nfev = ctypes.c_int64()
        njev = ctypes.c_int64()
        nobj = ctypes.c_int64()
        _check(self._lib.oi_cg_result(self._h, _ptr(x, ctypes.c_double), ctypes.byref(fun),
                                      ctypes.byref(nit), ctypes.byref(st), ctypes.byref(nfev),
                                      ctypes.byref(njev), ctypes.byref(nobj)))
        return dict(x=x, fun=fun.value, nit=nit.value, status=st.value, nfev=nfev.value,
                    njev=njev.value, nobj=nobj.value)

    def __del__(self):
        if getattr(self, '_h', None):
            self._lib.oi_cg_destroy(self._h)
            self._h = None


def _dptr(t, ctype=ctypes.c_double):
    """Device pointer of a torch tensor (plumbing for device_inputs=1 calls),
    after checking what liboi assumes: a contiguous CUDA tensor whose element
    type matches ``ctype`` (fp64 or int64, 8 bytes per element)."""
    want = {ctypes.c_double: 'torch.float64', ctypes.c_int64: 'torch.int64'}[ctype]
    if str(t.dtype) != want:
        raise ValueError(f"device array must be {want}, got {t.dtype}")
    if t.device.type != 'cuda':
        raise ValueError(f"device array must be a CUDA tensor, got {t.device}")
    if not t.is_contiguous():
        raise ValueError("device arrays must be contiguous")
    return ctypes.cast(t.data_ptr(), ctypes.POINTER(ctype))


def smooth_fields(fields, vmax, mask, kern, **opt_kw):
    """oi_smooth_fields (GPR:65-76 for nf fields): fields [nf, ny, nx] host
    arrays; kern the Gaussian2DKernel array (odd square).  Returns [nf, ny, nx]."""
    lib = load()
    f = np.ascontiguousarray(fields, dtype=np.float64)
    if f.ndim == 2:
        f = f[None]
    nf, ny, nx = f.shape
    vm = np.ascontiguousarray(np.broadcast_to(np.asarray(vmax, dtype=np.float64), (nf,)))
    m = np.ascontiguousarray(mask, dtype=np.float64)
    k = np.ascontiguousarray(kern, dtype=np.float64)
    if m.shape != (ny, nx) or k.ndim != 2 or k.shape[0] != k.shape[1] or k.shape[0] % 2 != 1:
        raise ValueError("mask must be [ny, nx] and kern an odd square")
    out = np.empty_like(f)
    _check(lib.oi_smooth_fields(_ptr(f, ctypes.c_double), nf, ny, nx, _ptr(vm, ctypes.c_double),
                                _ptr(m, ctypes.c_double), 0.0, _ptr(k, ctypes.c_double), k.shape[0],
                                _ptr(out, ctypes.c_double), ctypes.byref(options(**opt_kw))))
    return out


def smooth_fields_device(fields_dev, vmax, mask_dev, kern, out_dev, **opt_kw):
    """oi_smooth_fields on HBM-resident tensors ([nf, ny, nx] fp64 in and out)."""
    lib = load()
    nf, ny, nx = fields_dev.shape
    if tuple(mask_dev.shape) != (ny, nx) or tuple(out_dev.shape) != (nf, ny, nx):
        raise ValueError("shape mismatch")
    vm = np.ascontiguousarray(np.broadcast_to(np.asarray(vmax, dtype=np.float64), (nf,)))
    k = np.ascontiguousarray(kern, dtype=np.float64)
    _check(lib.oi_smooth_fields(_dptr(fields_dev), nf, ny, nx, _ptr(vm, ctypes.c_double),
                                _dptr(mask_dev), 0.0, _ptr(k, ctypes.c_double), k.shape[0],
                                _dptr(out_dev), ctypes.byref(options(device_inputs=True, **opt_kw))))
    return out_dev


def ball_query(pts, q, r, **opt_kw):
    """oi_ball_query on host arrays: returns (offs [Q+1], idx [offs[-1]])."""
    lib = load()
    P = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 2)
    Qa = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, 2)
    offs = np.zeros(len(Qa) + 1, dtype=np.int64)
    o = options(**opt_kw)
    _check(lib.oi_ball_query(_ptr(P, ctypes.c_double), len(P), _ptr(Qa, ctypes.c_double), len(Qa),
                             float(r), _ptr(offs, ctypes.c_int64), None, 0, ctypes.byref(o)))
    idx = np.empty(int(offs[-1]), dtype=np.int64)
    if len(idx):
        _check(lib.oi_ball_query(_ptr(P, ctypes.c_double), len(P), _ptr(Qa, ctypes.c_double),
                                 len(Qa), float(r), _ptr(offs, ctypes.c_int64),
                                 _ptr(idx, ctypes.c_int64), len(idx), ctypes.byref(o)))
    return offs, idx


def ball_query_device(pts_dev, q_dev, r, counts_only=False, **opt_kw):
    """oi_ball_query on HBM-resident [M, 2] / [Q, 2] tensors: returns
    (offs host [Q+1], idx device int64 tensor, or None with counts_only)."""
    import torch
    lib = load()
    M, Q = pts_dev.shape[0], q_dev.shape[0]
    offs = np.zeros(Q + 1, dtype=np.int64)
    o = options(device_inputs=True, **opt_kw)
    _check(lib.oi_ball_query(_dptr(pts_dev), M, _dptr(q_dev), Q, float(r),
                             _ptr(offs, ctypes.c_int64), None, 0, ctypes.byref(o)))
    if counts_only:
        return offs, None
    idx = torch.empty(int(offs[-1]), dtype=torch.int64, device=pts_dev.device)
    if idx.numel():
        _check(lib.oi_ball_query(_dptr(pts_dev), M, _dptr(q_dev), Q, float(r),
                                 _ptr(offs, ctypes.c_int64), _dptr(idx, ctypes.c_int64),
                                 idx.numel(), ctypes.byref(o)))
    return offs, idx


def gather_rows(x_train, y_train, t_train, z, idx, **opt_kw):
    """oi_gather_rows on host arrays: returns (xyt [N, 3], z [N])."""
    lib = load()
    cols = [np.ascontiguousarray(a, dtype=np.float64) for a in (x_train, y_train, t_train, z)]
    M = len(cols[0])
    if any(len(c) != M for c in cols):
        raise ValueError("training columns differ in length")
    I = np.ascontiguousarray(idx, dtype=np.int64)
    xyt = np.empty((len(I), 3))
    zo = np.empty(len(I))
    _check(lib.oi_gather_rows(*[_ptr(c, ctypes.c_double) for c in cols], M, _ptr(I, ctypes.c_int64),
                              len(I), _ptr(xyt, ctypes.c_double), _ptr(zo, ctypes.c_double),
                              ctypes.byref(options(**opt_kw))))
    return xyt, zo


def gather_rows_device(cols_dev, idx_dev, **opt_kw):
    """oi_gather_rows on HBM-resident tensors: cols_dev = (x, y, t, z) [M] each;
    returns (xyt [N, 3], z [N]) device tensors."""
    import torch
    lib = load()
    M = cols_dev[0].numel()
    N = idx_dev.numel()
    xyt = torch.empty((N, 3), dtype=torch.float64, device=idx_dev.device)
    zo = torch.empty(N, dtype=torch.float64, device=idx_dev.device)
    if N:
        _check(lib.oi_gather_rows(*[_dptr(c) for c in cols_dev], M, _dptr(idx_dev, ctypes.c_int64), N,
                                  _dptr(xyt), _dptr(zo),
                                  ctypes.byref(options(device_inputs=True, **opt_kw))))
    return xyt, zo


def profile_json():
    import json
    lib = load()
    n = lib.oi_profile_json(None, 0)
    buf = ctypes.create_string_buffer(int(n))
    lib.oi_profile_json(buf, n)
    return json.loads(buf.value.decode())


def profile_reset():
    load().oi_profile_reset()
