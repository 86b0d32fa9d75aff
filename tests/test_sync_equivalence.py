"""Equivalence oracle: every DP strategy yields the same weights.

Measured in the survey on CPU/gloo (N=4, B=16/rank, one SGD step): gather/
scatter, star p2p and DDP differ from per-param all-reduce by <=1.49e-8.
"""
import pytest
import torch

from mp_util import run_world

pytestmark = pytest.mark.slow


def _train(rank, world, mode, steps, opts):
    import torch.nn as nn
    from cs744_pytorch_distributed_tutorial_amd import distributed as D
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    from cs744_pytorch_distributed_tutorial_amd.parallel import DistributedDataParallel, make_comm, make_sync
    torch.manual_seed(5000)
    model = VGG11()
    if mode == "ddp":
        net = DistributedDataParallel(model, comm=make_comm("torch"), **opts)
        sync = make_sync("none", [])
    else:
        net = model
        sync = make_sync(mode, model.parameters(), group=D.new_group(list(range(world))), **opts)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    crit = nn.CrossEntropyLoss()
    g = torch.Generator().manual_seed(100 + rank)
    for _ in range(steps):
        x = torch.randn(8, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (8,), generator=g)
        opt.zero_grad()
        loss = crit(net(x), y)
        loss.backward()
        sync()
        opt.step()
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]), \
        torch.cat([b.detach().double().reshape(-1) for b in model.buffers()])


def _max_diff(a, b):
    return float((a - b).abs().max())


@pytest.mark.parametrize("world", [2, 4, 8])
def test_all_modes_agree(world):
    # N=8: one step. The modes differ only in the summation order of the averaged gradient
    # (~1e-8); from the second step on, that perturbs the forward, and at 64 samples a
    # pre-activation within rounding of 0 flips a ReLU mask often enough (measured: 8.9e-4
    # after two steps at N=8) that only the first step is a rounding-level oracle.
    steps = 1 if world == 8 else 2
    base = run_world(_train, world, "allreduce", steps, {})
    for r in range(1, world):
        assert _max_diff(base[r][0], base[0][0]) == 0.0  # replicas identical
    for mode, opts in [("gather_scatter", {}), ("p2p", {}), ("flat", {}), ("ddp", {}),
                       ("ddp", {"bucket_policy": "layer", "bucket_cap_mb": 4.0}),
                       ("gather_scatter", {"coalesce": True}), ("p2p", {"coalesce": True})]:
        res = run_world(_train, world, mode, steps, opts)
        for r in range(world):
            assert _max_diff(res[r][0], base[0][0]) < 1e-5, (mode, opts, r)
        for r in range(1, world):
            assert _max_diff(res[r][0], res[0][0]) < 1e-6, (mode, opts, r)


def _bn_prefwd(rank, world, broadcast):
    """Rank 1's BN buffers are pushed away from rank 0's; the buffers each rank's module sees
    at the START of its next training forward are captured by a forward pre-hook."""
    import torch.nn as nn
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    from cs744_pytorch_distributed_tutorial_amd.parallel import DistributedDataParallel, make_comm
    torch.manual_seed(5000)
    model = VGG11()
    net = DistributedDataParallel(model, comm=make_comm("torch"), broadcast_buffers=broadcast)
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(100 + rank)
    seen = []
    model.register_forward_pre_hook(
        lambda m, inp: seen.append(torch.cat([b.detach().double().reshape(-1) for b in m.buffers()])))
    for step in range(2):
        if step == 1 and rank == 1:
            with torch.no_grad():
                for b in model.buffers():
                    b.add_(3)  # rank-local drift: per-rank BN statistics (and any local edit)
        x = torch.randn(8, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (8,), generator=g)
        opt.zero_grad()
        nn.CrossEntropyLoss()(net(x), y).backward()
        opt.step()
    return seen[1]  # buffers entering the second training forward


def test_ddp_broadcasts_bn_buffers_from_rank0():
    """part3 DDP semantics (broadcast_buffers=True, `master/part3/part3.py:116`): every training
    forward starts from rank 0's BN buffers, so rank 1's drifted buffers are overwritten before
    its forward; the negative control (broadcast_buffers=False) keeps them apart."""
    res = run_world(_bn_prefwd, 2, True)
    assert torch.equal(torch.as_tensor(res[0]), torch.as_tensor(res[1]))
    off = run_world(_bn_prefwd, 2, False)
    assert _max_diff(torch.as_tensor(off[0]), torch.as_tensor(off[1])) >= 2.0


def test_single_process_differs_from_dp_due_to_per_rank_bn():
    """Non-equivalence guard: per-rank BN statistics make DP != large-batch single process."""
    import torch.nn as nn
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    res = run_world(_train, 2, "allreduce", 1, {})
    torch.manual_seed(5000)
    m = VGG11()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    xs, ys = [], []
    for r in range(2):
        g = torch.Generator().manual_seed(100 + r)
        xs.append(torch.randn(8, 3, 32, 32, generator=g))
        ys.append(torch.randint(0, 10, (8,), generator=g))
    opt.zero_grad()
    nn.CrossEntropyLoss()(m(torch.cat(xs)), torch.cat(ys)).backward()
    opt.step()
    single = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert _max_diff(single, res[0][0]) > 1e-5


def _eval_reduce(rank, world):
    from cs744_pytorch_distributed_tutorial_amd.parallel import make_comm
    from cs744_pytorch_distributed_tutorial_amd.utils.metrics import reduce_eval
    # rank r saw 10 + r test batches with 3 * r correct out of 64 * (10 + r), loss sum 2.0 per batch
    return reduce_eval(make_comm("torch"), 2.0 * (10 + rank), 3 * rank, 64 * (10 + rank), 10 + rank)


@pytest.mark.parametrize("world", [2, 4])
def test_global_accuracy_reduction(world):
    """The reference's intended cross-rank accuracy (its unmatched isend, C-4,
    `slave/part2b/part2b.py:67-69`): every rank gets the global (correct, total, mean loss)."""
    out = run_world(_eval_reduce, world)
    want_c = sum(3 * r for r in range(world))
    want_t = sum(64 * (10 + r) for r in range(world))
    for o in out:
        assert o["global_correct"] == want_c and o["global_total"] == want_t
        assert abs(o["global_avg_loss"] - 2.0) < 1e-12
