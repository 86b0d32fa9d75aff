"""CPU tests of the native engine's host-side logic: flat layout <-> reference
state_dict, block-aligned bucket plans, and the flat-buffer sync strategies over
a real multi-process gloo world (the same code drives RCCL on MI355X)."""
import math

import pytest
import torch

from mp_util import run_world


def test_layout_roundtrip_and_views():
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    torch.manual_seed(1)
    m = VGG11()
    for b in m.buffers():
        if b.dtype == torch.float32:
            b.uniform_()
        else:
            b.fill_(7)
    sd = m.state_dict()
    p = torch.zeros(lay.total)
    bufs = torch.zeros(lay.buf_total)
    nbt = torch.zeros(lay.L, dtype=torch.int64)
    lay.pack(sd, p, bufs, nbt)
    back = lay.unpack(p, bufs, nbt)
    assert list(back.keys()) == list(sd.keys()) and len(back) == 58
    for k in sd:
        assert torch.equal(back[k], sd[k]), k
    # every tensor 256-B aligned, padding is zero, sizes add up
    real = sum(v.numel() for v in m.parameters())
    assert real == 9_231_114
    assert all(off % 64 == 0 for off, _, _ in lay.entries.values())
    mask = torch.ones(lay.total, dtype=torch.bool)
    for off, n in lay.param_ranges():
        mask[off:off + n] = False
    assert p[mask].abs().sum() == 0
    # conv weights are stored OHWI (conv0 OIHW)
    off, shape, kind = lay.entries["layers.4.weight"]
    assert kind == "ohwi"
    assert torch.equal(p[off:off + math.prod(shape)].view(128, 3, 3, 64), sd["layers.4.weight"].permute(0, 2, 3, 1))
    assert lay.entries["layers.0.weight"][2] == "oihw"
    # backward-ready order: fc1 first, block 0 last
    assert lay.order[0] == "fc1.weight" and lay.order[-1] == "layers.1.bias"


@pytest.mark.parametrize("cap", [0.5, 4.0, 9.0, 25.0, 1e9])
def test_bucket_plan_is_contiguous_and_block_aligned(cap):
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    lows, ranges = lay.plan_buckets(cap)
    assert lows[-1] == 0 and lows == sorted(lows, reverse=True)
    pos = 0
    for off, n in ranges:
        assert off == pos
        pos = off + n
    assert pos == lay.total
    if cap >= 1e8:
        assert len(ranges) == 1
    if cap == 9.0:  # xGMI-sized: fc1+block7 | block6 | block5 | blocks 4..2 | small tail blocks 1..0
        assert lows == [7, 6, 5, 2, 0]
    if cap == 4.0:
        assert lows == [7, 6, 5, 4, 2, 0]  # b3+b2 | b1+b0 tail


def test_desc_chains():
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    for name in ("VGG11", "VGG13", "VGG16", "VGG19"):
        lay = FlatLayout(name)
        d = lay.desc()
        assert d[0] == 4 and d[2] == 32
        for l in range(1, lay.L):
            cin, cout, hw, pool = d[4 * l:4 * l + 4]
            pc, ph, pp = d[4 * (l - 1) + 1], d[4 * (l - 1) + 2], d[4 * (l - 1) + 3]
            assert cin == pc and hw == (ph // 2 if pp else ph)


def _flat_sync(rank, world, mode):
    from cs744_pytorch_distributed_tutorial_amd.parallel.comm import make_comm
    from cs744_pytorch_distributed_tutorial_amd.parallel.flat_sync import FlatGradSync
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    g = torch.Generator().manual_seed(10 + rank)
    flat = torch.zeros(lay.total)
    for off, n in lay.param_ranges():
        flat[off:off + n] = torch.randn(n, generator=g)
    FlatGradSync(mode, make_comm("torch"), lay.param_ranges(), lay.total)(flat)
    return flat


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 3])
def test_flat_sync_modes_agree(world):
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    expect = torch.zeros(lay.total)
    for r in range(world):
        g = torch.Generator().manual_seed(10 + r)
        for off, n in lay.param_ranges():
            expect[off:off + n] += torch.randn(n, generator=g)
    expect /= world
    for mode in ("allreduce", "gather_scatter", "p2p", "flat"):
        outs = run_world(_flat_sync, world, mode)
        for r in range(world):
            torch.testing.assert_close(outs[r], expect, rtol=1e-6, atol=1e-6, msg=f"{mode} rank {r}")
        assert all(torch.equal(outs[0], o) for o in outs[1:]), mode
