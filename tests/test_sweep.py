"""The 3D-1D sweep (BASELINE config 5, run_emi_3d1d.sh:5-17) sharded over
ranks (drivers.emi_3d1d_sweep): unit order, the shard partition, and the
gloo gather of a two-process run.  The solves here are stubs (host logic
only); tests/test_gpu_configs.py runs the real solves on the GPU in two
processes against the oracle's iteration counts."""
import os
import socket

import pytest


def _D():
    import metric_amg_examples_amd.drivers as D
    return D


def test_sweep_units_follow_the_script_loop():
    D = _D()
    u = D.sweep_units()
    assert len(u) == 24
    assert u[0] == (0.0, 1.0) and u[5] == (0.0, 1e10) and u[6] == (0.2, 1.0) and u[-1] == (5.0, 1e10)


@pytest.mark.parametrize('world', [1, 2, 3, 5, 8, 30])
def test_shards_partition_the_units(world):
    D = _D()
    units = D.sweep_units()
    seen = []
    for rank in range(world):
        part = D.shard_units(units, rank, world)
        assert all(k % world == rank for k, _ in part)
        assert all(units[k] == u for k, u in part)
        seen += [k for k, _ in part]
    assert sorted(seen) == list(range(len(units)))
    with pytest.raises(ValueError):
        D.shard_units(units, world, world)


def test_run_sweep_single_rank_and_lost_units():
    D = _D()
    units = D.sweep_units([0.0, 1.0], [1.0, 1e4])
    rows, wall, wmax = D.run_sweep(units, lambda u: dict(radius=u[0], gamma=u[1]))
    assert [(r['radius'], r['gamma']) for r in rows] == units
    assert wmax == wall
    with pytest.raises(RuntimeError):      # a gather that drops a rank's rows is an error, not a short table
        D.run_sweep(units, lambda u: {}, 0, 2, gather=lambda obj: [obj])


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import metric_amg_examples_amd.drivers as D

        def gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out
        units = D.sweep_units()
        rows, _, _ = D.run_sweep(units, lambda u: dict(radius=u[0], gamma=u[1], niters=int(u[0] * 10 + u[1] % 7)),
                                 rank, world, gather)
        q.put((rank, rows))
    finally:
        dist.destroy_process_group()


def test_sweep_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    D = _D()
    units = D.sweep_units()
    for rank in (0, 1):           # every rank holds the whole table, in the script's order
        rows = res[rank]
        assert [(r['radius'], r['gamma']) for r in rows] == units
        assert [r['rank'] for r in rows] == [k % 2 for k in range(len(units))]
