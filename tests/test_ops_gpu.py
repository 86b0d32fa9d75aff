"""Numerics of the gfx950 kernels vs plain PyTorch fp32 references (run on MI355X)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    native.C()  # must load: fail loudly otherwise
    return torch.device("cuda", 0)


@pytest.mark.parametrize("nhwc,cstride", [(False, 3), (True, 3), (True, 4)])
def test_augment_matches_reference(dev, nhwc, cstride):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    from cs744_pytorch_distributed_tutorial_amd.utils import data as dm
    ds = dm.SyntheticCIFAR10(train=True, size=300, seed=3)
    data = ds.data.to(dev)
    params = dm.augment_params(300, 0, 5, True).to(dev)
    idx = torch.randperm(300, device=dev)[:77]
    out = native.augment(data, idx, params, nhwc, cstride)
    ref = dm.augment_reference(data, idx, params, channels_last=nhwc)
    if nhwc and cstride == 4:
        assert torch.all(out[..., 3] == 0)
        out = out[..., :3]
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_augment_rejects_bad_index(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    data = torch.zeros(4, 32, 32, 3, dtype=torch.uint8, device=dev)
    params = torch.zeros(4, 3, dtype=torch.int32, device=dev)
    with pytest.raises(RuntimeError):
        native.augment(data, torch.tensor([5], device=dev), params)


@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_sgd_flat_matches_torch(dev, n):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.manual_seed(n)
    p0 = torch.randn(n, device=dev)
    grads = [torch.randn(n, device=dev) for _ in range(3)]
    ref = p0.clone().requires_grad_(False)
    rp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([rp], lr=0.1, momentum=0.9, weight_decay=1e-4)
    p, m = p0.clone(), torch.zeros(n, device=dev)
    for i, g in enumerate(grads):
        rp.grad = g.clone()
        opt.step()
        native.sgd_flat(p, g, m, 0.1, 0.9, 1e-4, 0.0, 1.0, i == 0)
    torch.testing.assert_close(p, rp.detach(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(m, opt.state[rp]["momentum_buffer"], rtol=1e-6, atol=1e-6)


def test_fused_sgd_optimizer_matches_torch(dev):
    from cs744_pytorch_distributed_tutorial_amd.models import VGG11
    from cs744_pytorch_distributed_tutorial_amd.ops.optim import FusedSGD
    torch.manual_seed(0)
    a, b = VGG11().to(dev), VGG11().to(dev)
    b.load_state_dict(a.state_dict())
    oa = torch.optim.SGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    ob = FusedSGD(b.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    for s in range(3):
        for pa, pb in zip(a.parameters(), b.parameters()):
            g = torch.randn_like(pa)
            pa.grad, pb.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-6, atol=1e-6)
    # identical checkpoint format
    assert set(oa.state_dict()["state"].keys()) == set(ob.state_dict()["state"].keys())


@pytest.mark.parametrize("B", [1, 20, 64, 256])
def test_linear_xent_matches_torch(dev, B):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.manual_seed(B)
    feat = torch.randn(B, 512, device=dev, requires_grad=True)
    W = (torch.randn(10, 512, device=dev) * 0.05).requires_grad_()
    bias = torch.randn(10, device=dev, requires_grad=True)
    y = torch.randint(0, 10, (B,), device=dev)
    logits = torch.nn.functional.linear(feat, W, bias)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    out = native.linear_xent(feat.detach(), W.detach(), bias.detach(), y, 1.0, True)
    l, correct, lg, dW, db, dfeat, pred = out
    torch.testing.assert_close(l, loss.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(lg, logits.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dW, W.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(db, bias.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dfeat, feat.grad, rtol=1e-4, atol=1e-6)
    assert int(correct) == int((logits.argmax(1) == y).sum())
    torch.testing.assert_close(pred, logits.argmax(1))


def test_softmax_xent_matches_torch(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    lg = torch.randn(64, 10, device=dev, requires_grad=True)
    y = torch.randint(0, 10, (64,), device=dev)
    loss = torch.nn.functional.cross_entropy(lg, y)
    loss.backward()
    l, dl, c = native.softmax_xent(lg.detach(), y)
    torch.testing.assert_close(l, loss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dl, lg.grad, rtol=1e-5, atol=1e-7)


def test_flat_sync_root_combines_match_torch(dev):
    """part2a / part2a_extra root combines on the flat buffer (flat_ops.hip) vs ATen."""
    from cs744_pytorch_distributed_tutorial_amd import _C
    torch.manual_seed(3)
    for w, n in ((2, 1), (4, 1003), (8, 65536 + 3)):
        src = torch.randn(w * n, device="cuda")
        dst = torch.empty(n, device="cuda")
        _C.rows_mean(src, w, dst)
        ref = src.view(w, n).double().mean(0).float()
        torch.testing.assert_close(dst, ref, rtol=1e-6, atol=1e-7)
        rows = src.clone()
        dst2 = torch.empty(n, device="cuda")
        _C.rows_mean(rows, w, dst2, True)  # the mean also over every row: the scatter list
        assert torch.equal(dst2, dst) and torch.equal(rows.view(w, n), dst.expand(w, n))
        g = torch.randn(n, device="cuda")
        ts = [torch.randn(n, device="cuda") for _ in range(w - 1)]
        exp = g.clone()
        for i, t in enumerate(ts):
            _C.accumulate(g, t, float(w) if i == len(ts) - 1 else 0.0)
            exp.add_(t)
        exp.div_(w)
        assert torch.equal(g, exp)
