"""The framework DDP (parallel/ddp.py) over a ONE-RANK native RcclComm on the MI355X — the exact
data plane the ResNet-50 / Llama-3-8B extension configs use at N > 1 (bucketed all-reduce(AVG)
forked onto the comm stream from the backward's hooks, joined before the optimizer) — must
reproduce the no-DDP step: bitwise with fp32 transport (an average over one rank is exact), to
bf16 rounding with the bf16 transport; plus the bf16 cast kernels themselves."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    native.C()
    return torch.device("cuda", 0)


def _run(dev, model, ddp, gdt=None, steps=3):
    from cs744_pytorch_distributed_tutorial_amd.parallel import DistributedDataParallel
    from cs744_pytorch_distributed_tutorial_amd.parallel.rccl import RcclComm
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import build_model
    torch.manual_seed(0)
    m = build_model(model).to(dev)
    is_lm = hasattr(m, "vocab_size")
    g = torch.Generator(device="cpu").manual_seed(1)
    if is_lm:
        data = [torch.randint(0, m.vocab_size, (2, 65), generator=g).to(dev) for _ in range(steps)]
    else:
        m = m.to(memory_format=torch.channels_last)
        data = [(torch.randn(4, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last),
                 torch.randint(0, 1000, (4,), generator=g).to(dev)) for _ in range(steps)]
    comm = RcclComm.create(0, 1, dev.index or 0, max_ctas=8) if ddp else None
    net = DistributedDataParallel(m, comm=comm, bucket_cap_mb=1.0, grad_comm_dtype=gdt) if ddp else m
    opt = torch.optim.SGD(net.parameters(), lr=0.01, momentum=0.9)
    for d in data:
        opt.zero_grad()
        if is_lm:
            logits = net(d[:, :-1])
            loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, m.vocab_size), d[:, 1:].reshape(-1))
        else:
            loss = torch.nn.functional.cross_entropy(net(d[0]).float(), d[1])
        loss.backward()
        opt.step()
    torch.cuda.synchronize()
    if ddp:
        assert comm.native.calls() > 0 and comm.native.max_ctas == 8
    return torch.cat([p.detach().float().reshape(-1) for p in m.parameters()])


@pytest.mark.parametrize("model", ["resnet18", "llama-tiny"])
def test_ddp_over_one_rank_rccl_equals_plain_step(dev, model):
    ref = _run(dev, model, ddp=False)
    got = _run(dev, model, ddp=True)
    assert torch.equal(ref, got)


@pytest.mark.parametrize("model", ["resnet18", "llama-tiny"])
def test_ddp_bf16_transport_one_rank(dev, model):
    """One SGD step: each weight moves by lr * g in both runs, with g rounded once to bf16 on the
    wire in one of them (round to nearest: relative error <= half an ulp = 2^-8), so |difference| <=
    2^-8 |g| lr <= 2^-8 * the largest update (later steps would compound the rounding through BN's
    batch statistics)."""
    ref = _run(dev, model, ddp=False, steps=1)
    p0 = _run(dev, model, ddp=False, steps=0)
    got = _run(dev, model, ddp=True, gdt=torch.bfloat16, steps=1)
    upd = (ref - p0).abs().max()
    assert 0 < (got - ref).abs().max() <= 2.0 ** -8 * upd * 1.01


def test_cast_grad_kernels(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    x = torch.randn(100003, device=dev) * torch.logspace(-30, 30, 100003, device=dev)
    x[7] = float("nan")
    x[8] = float("inf")
    b = torch.empty(x.numel(), device=dev, dtype=torch.bfloat16)
    C.cast_grad(x, b)
    ref = x.bfloat16()
    assert torch.equal(b.view(torch.int16)[~ref.isnan()], ref.view(torch.int16)[~ref.isnan()])
    assert b[7].isnan()
    back = torch.empty_like(x)
    C.cast_grad(b, back)
    assert torch.equal(back[~back.isnan()], ref.float()[~back.isnan()])
