"""Config 4's code path on the real HIP library: two ranks (one process each)
sharing cuda:0, collectives over gloo on the host (the 1-GPU box cannot run
RCCL between two processes on one device).  The reference distributes cells
over MPI ranks (split GPR:18-23, scatter GPR:256) and gathers per-cell tuples
(GPR:262, GPR:320); cells are independent and per-cell arithmetic never
depends on the batch, so the sharded results must equal the single-rank
call BITWISE:
  * driver.run_sharded(..., driver.gpu_compute())  (pass 1, LPT partition)
  * day.interpolate_day(world=2)                   (two-pass day pipeline:
    device neighbour query, pass 1, all_gather, smoothing, pass 2, gather)
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

X0 = np.array([np.log(25e3), np.log(25e3), 0.0, 0.0, 0.0, np.log(.1)])


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cells():
    from optimalinterpolation_amd import synthetic
    return synthetic.make_cells(np.random.default_rng(3).integers(30, 260, 300), seed=17)


def _binned_day():
    from optimalinterpolation_amd import synthetic
    return synthetic.make_binned_day(seed=8, nx=40, ice_radius_m=120e3, obs_radius_m=450e3,
                                     cover=(0.02, 0.05))


def _worker(rank, world, port, q, logpath):
    import faulthandler
    import traceback
    log = open(logpath, 'a', buffering=1)
    faulthandler.dump_traceback_later(60, repeat=False, file=log)  # where a hung rank sits
    try:
        import torch
        import torch.distributed as dist
        from optimalinterpolation_amd import day, driver
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        log.write(f"rank {rank}: process group up\n")
        torch.cuda.set_device(0)
        full = driver.run_sharded(_cells(), driver.gpu_compute(opt=True, x0=X0, device=0), rank, world)
        log.write(f"rank {rank}: run_sharded done\n")
        d = _binned_day()
        res = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d', rank=rank, world=world,
                                  device=0, comm_device=torch.device('cpu'))
        log.write(f"rank {rank}: interpolate_day done\n")
        q.put((rank, full, None if res is None else {k: np.asarray(v) for k, v in res.items()}, None))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        q.put((rank, None, None, traceback.format_exc()))
        raise


def test_two_ranks_equal_one_rank_bitwise(tmp_path):
    import queue
    import time
    from optimalinterpolation_amd import _lib, day
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    logpath = str(tmp_path / 'ranks.log')
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, logpath)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    deadline = time.time() + 150
    try:
        while len(got) < world:
            try:
                r, full, res, err = q.get(timeout=2)
            except queue.Empty:
                dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
                log = open(logpath).read() if os.path.exists(logpath) else ''
                assert not dead and time.time() < deadline, f"ranks failed/hung: exit {dead}\n{log}"
                continue
            assert err is None, f"rank {r} raised:\n{err}"
            got[r] = (full, res)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert got[1][0] is None and got[1][1] is None  # only rank 0 holds the gathered results
    full, res = got[0]
    # single rank, same library, same cells
    cells = _cells()
    out, st, info = _lib.gpr_batch(cells.xyt, cells.z, cells.offs, cells.xs, cells.mean, x0=X0, opt=True,
                                   info=True)
    assert full.shape == (cells.ncell, 13)
    assert np.array_equal(full[:, :8], out, equal_nan=True)
    assert np.array_equal(full[:, 8], st.astype(float))
    assert np.array_equal(full[:, 9:], info.astype(float))
    d = _binned_day()
    ref = day.interpolate_day(d.sat, d.sie, d.x, d.y, d.mean, date='d')
    assert set(res) == set(ref)
    for k in ref:
        assert np.array_equal(res[k], np.asarray(ref[k]), equal_nan=True), k


def test_bench_self_launch_gloo(tmp_path):
    """`python bench.py --gpus 2` with no launcher around it (VERDICT r4 item
    1): bench.py starts both ranks itself, they shard a (shortened) day over
    one GPU with gloo collectives, and rank 0's line reports the world."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / 'line.json'
    env = dict(os.environ, OI_DIST_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '4',
                        '--warmup', '1', '--day-cells', '96', '--no-cpu-baseline', '--parity-cells', '4',
                        '--budget-s', '90', '--out', str(out)],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line == json.loads(out.read_text())
    assert line['n_gpus'] == 2 and line['ranks_seen'] == [0, 1] and line['rank_devices'] == [0, 0]
    assert line['collective_backend'] == 'gloo' and line['launcher'] == 'bench.py'
    assert line['config']['cells_total'] == 96 and line['failed_cells'] == 0
    assert line['steps'] == 4 and not line.get('truncated')
    assert line['parity']['pass'], line['parity']
    # per-rank evidence: both ranks, their cells summing to the day
    pr = line['per_rank']
    assert [r['rank'] for r in pr] == [0, 1] and sum(r['cells'] for r in pr) == 96
    assert line['config']['cells_per_rank'] == [r['cells'] for r in pr]
    assert all(0 < r['own_work_s'] <= line['timed_s'] + 1e-3 and r['evals'] > 0 for r in pr)


def test_bench_under_torchrun_gloo(tmp_path):
    """The driver's N > 1 launch shape, `python -m torch.distributed.run
    --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P
    bench.py --gpus N ...`: WORLD_SIZE comes from the launcher, bench.py starts
    no ranks of its own, and the line reports the launcher (two gloo ranks
    sharing the one GPU of this box)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / 'line.json'
    env = dict(os.environ, OI_DIST_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT', 'OI_BENCH_LAUNCHER'):
        env.pop(k, None)
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
                        os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '4', '--warmup', '1',
                        '--day-cells', '96', '--no-cpu-baseline', '--parity-cells', '4', '--budget-s', '90',
                        '--out', str(out)],
                       env=env, capture_output=True, text=True, timeout=110, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line['n_gpus'] == 2 and line['ranks_seen'] == [0, 1] and line['rank_devices'] == [0, 0]
    assert line['collective_backend'] == 'gloo' and line['launcher'] == 'torch.distributed.run'
    assert line['config']['cells_total'] == 96 and line['failed_cells'] == 0
    assert line['steps'] == 4 and not line.get('truncated')
    assert line['parity']['pass'], line['parity']


def test_bench_twopass_small(tmp_path):
    """`bench.py --workload twopass` (the reference's whole two-pass day,
    GPR:223-336) end to end on a small binned day: the line's parity block
    (smoothing bit-exact vs the oracle on the GPU's own pass-1 fields, pass-2
    cells at T1) passes and the stages add up."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / 'twopass.json'
    p = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), '--workload', 'twopass', '--twopass-small',
                        '--steps', '1', '--no-cpu-baseline', '--parity-cells', '6', '--out', str(out)],
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(out.read_text())
    assert line['parity']['pass'], line['parity']
    assert all(line['parity']['smooth_bit_exact'])
    st = line['stages_s']
    assert st['pass1_s'] > 0 and st['pass2_s'] > 0 and st['total_s'] >= st['pass1_s'] + st['pass2_s']
    assert line['failed_cells'] == 0 and line['config']['day_cells'] > 20
