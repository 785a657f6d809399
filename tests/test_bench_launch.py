"""bench.py's own rank launcher (VERDICT r4 "next" item 1): `python bench.py
--gpus N` with no launcher around it starts N rank processes with the
torch.distributed.run environment contract, forwards rank 0's JSON line and
fails loudly.  Checked on the CPU with a stand-in rank script (the GPU leg
itself is `tests/test_gpu_multirank.py::test_bench_self_launch_gloo`)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = textwrap.dedent('''
    import json, os, sys, time
    mode = sys.argv[1]
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                          "MASTER_ADDR", "MASTER_PORT", "OI_BENCH_LAUNCHER", "OI_BENCH_T0")}
    r = int(env["RANK"])
    if mode == "fail1" and r == 1:
        sys.exit(7)
    if mode == "fail1":
        time.sleep(120)          # the launcher must end this rank
    if mode == "noline":
        sys.exit(0)
    if mode == "stuck0":         # rank 1 exits 0, rank 0 hangs (e.g. in a collective)
        if r == 1:
            sys.exit(0)
        time.sleep(120)
    if mode == "dist":
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = [torch.zeros(1) for _ in range(int(env["WORLD_SIZE"]))]
        dist.all_gather(t, torch.tensor([float(r)]))
        env["seen"] = [int(x.item()) for x in t]
        dist.destroy_process_group()
    if r == 0:
        print("not json", flush=True)
        print(json.dumps(env), flush=True)
''')


@pytest.fixture
def rank_script(tmp_path):
    p = tmp_path / 'rank.py'
    p.write_text(RANK_SCRIPT)
    return str(p)


def test_launch_sets_the_rank_environment_and_forwards_rank0_line(rank_script, capfd):
    rc = bench.launch_ranks(3, ['ok'], script=rank_script, gpus=8, backend='nccl')
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    env = json.loads(out[-1])
    assert env['RANK'] == '0' and env['LOCAL_RANK'] == '0'
    assert env['WORLD_SIZE'] == '3' and env['LOCAL_WORLD_SIZE'] == '3'
    assert env['MASTER_ADDR'] == '127.0.0.1' and int(env['MASTER_PORT']) > 0
    assert env['OI_BENCH_LAUNCHER'] == 'bench.py'
    assert abs(float(env['OI_BENCH_T0']) - bench.T_PROC) < 1e-6


def test_launched_ranks_rendezvous(rank_script, capfd):
    rc = bench.launch_ranks(2, ['dist'], script=rank_script, gpus=2, backend='gloo')
    assert rc == 0
    env = json.loads(capfd.readouterr().out.strip().splitlines()[-1])
    assert env['seen'] == [0, 1]


def test_failing_rank_ends_the_others_and_sets_the_exit_code(rank_script):
    t0 = time.time()
    rc = bench.launch_ranks(3, ['fail1'], script=rank_script, gpus=8, backend='nccl', grace_s=5.0)
    assert rc == 7
    assert time.time() - t0 < 60          # rank 0 / 2 (sleeping 120 s) were ended, not waited for


def test_launcher_deadline_ends_a_stuck_rank(rank_script):
    """a rank stuck after another exited 0 is ended at the deadline."""
    t0 = time.time()
    rc = bench.launch_ranks(2, ['stuck0'], script=rank_script, gpus=8, backend='nccl', grace_s=5.0,
                            deadline_s=bench.elapsed() + 8.0)
    assert rc == 124
    assert time.time() - t0 < 60


def test_rank0_without_a_line_is_a_failure(rank_script):
    assert bench.launch_ranks(2, ['noline'], script=rank_script, gpus=8, backend='nccl') == 1


def test_oversubscription_is_refused_unless_gloo(rank_script):
    assert bench.launch_ranks(2, ['ok'], script=rank_script, gpus=1, backend='nccl') == 2
    assert bench.launch_ranks(2, ['ok'], script=rank_script, gpus=1, backend='gloo') == 0


def test_world_size_must_equal_gpus():
    env = dict(os.environ, WORLD_SIZE='2', RANK='0', LOCAL_RANK='0')
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '1', '--no-cpu-baseline'],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and 'misreport n_gpus' in p.stderr


def _args(**kw):
    import argparse
    a = dict(workload='day', day_shares=0, share=-1)
    a.update(kw)
    return argparse.Namespace(**a)


def test_share_arguments_are_validated():
    with pytest.raises(SystemExit):
        bench.check_shares(_args(share=3), 1, 1)            # --share without --day-shares
    with pytest.raises(SystemExit):
        bench.check_shares(_args(share=8, day_shares=8), 1, 8)
    with pytest.raises(SystemExit):
        bench.check_shares(_args(share=0, day_shares=8), 8, 8)  # --share with N ranks
    with pytest.raises(SystemExit):
        bench.check_shares(_args(day_shares=16), 8, 16)     # shares 8..15 never fitted
    bench.check_shares(_args(share=7, day_shares=8), 1, 8)
    bench.check_shares(_args(day_shares=8), 8, 8)


def test_default_depth_depends_on_the_per_rank_work_not_the_gpu_count():
    # a whole day per rank: 8 at any N; a share of a day: every slice at any N
    for world in (1, 2, 8):
        assert bench.default_depth(_args(workload='days'), world, 20)[0] == 8
        assert bench.default_depth(_args(workload='season'), world, 20)[0] == 20
    assert bench.default_depth(_args(workload='day'), 1, 20)[0] == 8
    assert bench.default_depth(_args(workload='day', day_shares=8), 1, 20)[0] == 20
    assert bench.default_depth(_args(workload='day'), 8, 20)[0] == 20
    # the season: keyed on one day's slices, not every slice of K days
    assert bench.default_depth(_args(workload='season'), 1, 60, [20, 20, 20])[0] == 20
