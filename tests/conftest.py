import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    # pytest-xdist workers: one BLAS thread each.  Several workers each running
    # a full OpenBLAS thread pool on the same CPUs turn the oracle's many small
    # solves into spin-wait contention (test_cg_trace_bitwise: 4.5 s alone,
    # 640 s under -n 4).  The bitwise golden checks (tests/test_oracle_golden.py,
    # test_day_two_ranks_equals_one) were made with OpenBLAS's default thread
    # count and do not hold at one thread: they are marked `blas_default` and
    # run with the default count restored (fixture below).
    config.addinivalue_line("markers", "blas_default: needs OpenBLAS's default thread count (bitwise goldens)")
    if os.environ.get('PYTEST_XDIST_WORKER'):
        try:
            from threadpoolctl import threadpool_info, threadpool_limits
            global _BLAS_DEFAULT
            _BLAS_DEFAULT = max((d.get('num_threads', 1) for d in threadpool_info()), default=None)
            threadpool_limits(1)
        except ImportError:
            pass


_BLAS_DEFAULT = None


@pytest.fixture(autouse=True)
def _blas_default_threads(request):
    if _BLAS_DEFAULT is None or request.node.get_closest_marker('blas_default') is None:
        yield
        return
    from threadpoolctl import threadpool_limits
    # one such test at a time across the workers: two full OpenBLAS pools on
    # the same CPUs spin against each other (test_gpr3d_bitwise: 9 s alone,
    # ~575 s beside test_cg_trace_bitwise under -n 4)
    try:
        from filelock import FileLock
        lock = FileLock(os.path.join(os.environ.get('TMPDIR', '/tmp'), 'oi_blas_default_tests.lock'))
    except ImportError:
        import contextlib
        lock = contextlib.nullcontext()
    with lock, threadpool_limits(_BLAS_DEFAULT):
        yield


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def ragged_cell(d, c, xkey='x', ykey='y', okey='offs'):
    a, b = int(d[okey][c]), int(d[okey][c + 1])
    return d[xkey][a:b].reshape(-1, 3), d[ykey][a:b]


@pytest.fixture(scope='session')
def golden():
    return load_golden
