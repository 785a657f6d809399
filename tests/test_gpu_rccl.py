"""The RCCL ('nccl') collective path on the GPU box.  A one-GPU box cannot
hold two RCCL ranks (RCCL refuses two ranks on one device), so the
multi-rank tests rehearse over gloo; here a one-rank RCCL process group runs
the exact device-tensor collectives of the sharded pass -- the LPT partition,
the batched liboi call and driver.gather_rows' single gather / all_gather of
the ncell x 13 rows, payload in HBM -- and the result must equal the plain
batched call bitwise (GPR:256-262's scatter / gather)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

X0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])


def test_rccl_one_rank_sharded_pass_equals_plain_call():
    import torch
    import torch.distributed as dist
    from optimalinterpolation_amd import _lib, driver, synthetic
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1,
                            device_id=torch.device('cuda', 0))
    try:
        assert dist.get_backend() == 'nccl'
        cells = synthetic.make_cells(np.random.default_rng(4).integers(30, 400, 40), seed=19)
        dev = torch.device('cuda', 0)
        full = driver.run_sharded(cells, driver.gpu_compute(opt=True, x0=X0, device=0), 0, 1, device=dev)
        rows = np.arange(cells.ncell * 3, dtype=np.float64).reshape(cells.ncell, 3)
        both = driver.gather_rows(rows, [np.arange(cells.ncell)], cells.ncell, device=dev, to_all=True)
    finally:
        dist.destroy_process_group()
    out, st, info = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True,
                                   info=True)
    assert np.array_equal(full[:, :8], out, equal_nan=True)
    assert np.array_equal(full[:, 8], st.astype(float)) and np.array_equal(full[:, 9:], info.astype(float))
    assert np.array_equal(both, rows)
