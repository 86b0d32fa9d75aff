"""Facade semantics on a real multi-process gloo world (SURVEY.md §4.2 'Unit, comm (CPU)')."""
import pytest
import torch

from mp_util import run_world

pytestmark = pytest.mark.slow


def _api(rank, world):
    from cs744_pytorch_distributed_tutorial_amd import distributed as D
    out = {}
    assert D.get_rank() == rank and D.get_world_size() == world
    # reference hard-codes new_group([0,1,2,3]); it must work at any world size
    g = D.new_group([0, 1, 2, 3])
    t = torch.full((5,), float(rank + 1))
    D.all_reduce(t, op=D.reduce_op.SUM, group=g)
    out["sum"] = t.tolist()
    t = torch.full((3,), float(rank))
    D.all_reduce(t, op=D.ReduceOp.AVG)
    out["avg"] = t.tolist()
    # gather / scatter as in part2a
    g_in = torch.full((4,), float(rank))
    lst = [torch.zeros(4) for _ in range(world)] if rank == 0 else None
    D.gather(g_in, lst, dst=0)
    if rank == 0:
        out["gathered"] = [x.tolist() for x in lst]
    s = torch.zeros(2)
    D.scatter(s, [torch.full((2,), 10.0 + r) for r in range(world)] if rank == 0 else None, src=0)
    out["scattered"] = s.tolist()
    # broadcast + barrier
    b = torch.tensor([7.0 if rank == 0 else -1.0])
    D.broadcast(b, src=0)
    out["bcast"] = b.item()
    D.barrier()
    # p2p ring with isend/irecv + wait
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    sbuf = torch.tensor([float(rank)])
    rbuf = torch.zeros(1)
    if rank % 2 == 0:
        D.isend(sbuf, dst=nxt).wait()
        D.irecv(rbuf, src=prv).wait()
    else:
        D.irecv(rbuf, src=prv).wait()
        D.isend(sbuf, dst=nxt).wait()
    out["ring"] = rbuf.item()
    # async AVG on gloo goes through SUM + scale
    a = torch.full((4,), float(rank))
    w = D.all_reduce(a, op=D.ReduceOp.AVG, async_op=True)
    w.wait()
    out["async_avg"] = a.tolist()
    out["scalar"] = D.all_reduce_scalar(float(rank))
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_facade_collectives(world):
    res = run_world(_api, world)
    s = sum(range(1, world + 1))
    mean = sum(range(world)) / world
    for r, o in enumerate(res):
        assert o["sum"] == [float(s)] * 5
        assert o["avg"] == pytest.approx([mean] * 3)
        assert o["scattered"] == [10.0 + r] * 2
        assert o["bcast"] == 7.0
        assert o["ring"] == float((r - 1) % world)
        assert o["async_avg"] == pytest.approx([mean] * 4)
        assert o["scalar"] == sum(range(world))
    assert res[0]["gathered"] == [[float(r)] * 4 for r in range(world)]


def _pingpong(rank, world):
    from cs744_pytorch_distributed_tutorial_amd.entrypoints.part1_pingpong import pingpong
    return pingpong([8, 4096, 1 << 20], iters=3, warmup=1, use_async=(rank >= 0))


def test_pingpong_world2():
    res = run_world(_pingpong, 2)
    assert len(res[0]) == 3 and all(r["rtt_us"] > 0 for r in res[0])
    assert res[1] == []
