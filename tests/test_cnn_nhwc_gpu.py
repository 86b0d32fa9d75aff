"""Channels-last CNN path (csrc/kernels/cnn_nhwc.hip, ops/cnn_nhwc.py) against plain PyTorch
fp64/fp32 references: convolution through im2col + GEMM (forward, data and weight gradients)
for every geometry ResNet uses, training BatchNorm (+residual) (+ReLU) with running statistics,
the 3x3/2 max-pool, bitwise run-to-run determinism, and a whole ResNet-18 step against the
NCHW module path."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    native.C()
    return torch.device("cuda", 0)


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2)


# (B, Cin, H, W, Cout, k, stride, pad): every ResNet geometry (stem, 1x1, strided 1x1, 3x3, 3x3/2)
CONVS = [(2, 3, 32, 32, 16, 7, 2, 3), (2, 16, 14, 14, 32, 1, 1, 0), (2, 16, 14, 14, 32, 1, 2, 0),
         (3, 8, 9, 11, 16, 3, 1, 1), (2, 32, 14, 14, 16, 3, 2, 1), (1, 4, 5, 5, 8, 3, 1, 1),
         (8, 16, 32, 32, 16, 3, 1, 1), (16, 8, 32, 32, 32, 1, 1, 0)]  # the last two: split weight-gradient GEMM


@pytest.mark.parametrize("geo", CONVS)
def test_conv_nhwc_matches_fp64(dev, geo):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import conv_nhwc
    B, Ci, H, W, Co, k, st, pad = geo
    torch.manual_seed(sum(geo))
    conv = nn.Conv2d(Ci, Co, k, stride=st, padding=pad, bias=False).to(dev)
    x = torch.randn(B, Ci, H, W, device=dev)
    xh = nhwc(x).requires_grad_()
    y = conv_nhwc(xh, conv)
    xr = x.double().requires_grad_()
    wr = conv.weight.detach().double().requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pad)
    torch.testing.assert_close(nchw(y).double(), yr, rtol=1e-4, atol=1e-4)
    g = torch.randn(yr.shape, device=dev)
    y.backward(nhwc(g))
    yr.backward(g.double())
    torch.testing.assert_close(nchw(xh.grad).double(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(conv.weight.grad.double(), wr.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_nhwc_padded_stem(dev, dtype):
    """the stem's 3-channel weight on a 4-channel input whose last channel is zero (vector im2col)"""
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import conv_nhwc, to_nhwc
    torch.manual_seed(7)
    conv = nn.Conv2d(3, 16, 7, stride=2, padding=3, bias=False).to(dev)
    x = torch.randn(2, 3, 40, 40, device=dev)
    xh = to_nhwc(x, dtype, pad_c=1)
    assert xh.shape == (2, 40, 40, 4) and bool((xh[..., 3] == 0).all())
    y = conv_nhwc(xh, conv)
    wr = conv.weight.detach().to(dtype).double().requires_grad_()
    yr = F.conv2d(x.to(dtype).double(), wr, None, 2, 3)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(nchw(y).double(), yr, **tol)
    g = torch.randn(yr.shape, device=dev)
    y.backward(nhwc(g).to(dtype))
    yr.backward(g.to(dtype).double())
    assert conv.weight.grad.shape == (16, 3, 7, 7) and conv.weight.grad.is_contiguous()
    torch.testing.assert_close(conv.weight.grad.double(), wr.grad, rtol=1e-4 if dtype == torch.float32 else 2e-2,
                               atol=1e-3 if dtype == torch.float32 else 0.5)


def test_conv_nhwc_bf16_close(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import conv_nhwc
    torch.manual_seed(3)
    conv = nn.Conv2d(64, 64, 3, padding=1, bias=False).to(dev)
    x = torch.randn(4, 64, 14, 14, device=dev)
    xh = nhwc(x).bfloat16().requires_grad_()
    y = conv_nhwc(xh, conv)
    assert y.dtype == torch.bfloat16
    yr = F.conv2d(xh.detach().float().permute(0, 3, 1, 2), conv.weight.bfloat16().float(), None, 1, 1)
    torch.testing.assert_close(nchw(y).float(), yr, rtol=2e-2, atol=3e-2)
    y.float().square().sum().backward()
    assert conv.weight.grad.dtype == torch.float32 and torch.isfinite(conv.weight.grad).all()


@pytest.mark.parametrize("shape", [(4, 56, 56, 64), (8, 7, 7, 2048), (3, 14, 14, 24), (2, 5, 3, 6), (64, 3, 3, 512)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_bn_act_nhwc_matches_fp64(dev, shape, dtype, relu, residual):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import bn_act_nhwc
    torch.manual_seed(hash((shape, relu, residual)) % 1000)
    C = shape[3]
    bn = nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
    rm0, rv0 = bn.running_mean.clone().double(), bn.running_var.clone().double()
    x = (torch.randn(shape, device=dev) * 2 + 0.7).to(dtype).requires_grad_()
    res = torch.randn(shape, device=dev).to(dtype).requires_grad_() if residual else None
    y = bn_act_nhwc(bn, x, relu, res)
    assert y.shape == x.shape and y.dtype == dtype
    xr = x.detach().double().requires_grad_()
    rr = res.detach().double().requires_grad_() if residual else None
    wr = bn.weight.detach().double().requires_grad_()
    br = bn.bias.detach().double().requires_grad_()
    yr = F.batch_norm(nchw(xr), rm0.clone(), rv0.clone(), wr, br, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    if residual:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.double(), yr, **tol)
    xd = x.detach().double().reshape(-1, C)
    M = xd.shape[0]
    torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0 + 0.1 * xd.mean(0), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), 0.9 * rv0 + 0.1 * xd.var(0, unbiased=M > 1), rtol=1e-4,
                               atol=1e-5)
    assert int(bn.num_batches_tracked) == 1
    g = torch.randn(shape, device=dev).to(dtype)
    y.backward(g)
    yr.backward(g.double())
    gt = dict(rtol=1e-3, atol=1e-3) if dtype == torch.float32 else dict(rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.double(), xr.grad, **gt)
    pt = dict(rtol=1e-3, atol=1e-2 if dtype == torch.bfloat16 else 1e-3)
    torch.testing.assert_close(bn.weight.grad.double(), wr.grad, **pt)
    torch.testing.assert_close(bn.bias.grad.double(), br.grad, **pt)
    if residual:
        torch.testing.assert_close(res.grad.double(), rr.grad, **gt)


@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 9, 7, 24), (2, 5, 6, 6)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_maxpool_fused_equals_two_passes(dev, shape, dtype, monkeypatch):
    """the stem's BatchNorm + ReLU + 3x3/2 max-pool with the apply fused into the pool is bitwise equal
    to the separate passes (CS_BN_POOL_FUSE=0): output, input / weight / bias gradients and running
    statistics"""
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import bn_relu_maxpool_nhwc
    torch.manual_seed(8)
    x0 = torch.randn(shape, device=dev).to(dtype)
    outs = []
    for m in ("0", "1"):
        monkeypatch.setenv("CS_BN_POOL_FUSE", m)
        bn = nn.BatchNorm2d(shape[3]).to(dev)
        torch.manual_seed(10)  # the same affine parameters for every run
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        x = x0.clone().requires_grad_()
        y = bn_relu_maxpool_nhwc(bn, x)
        g = torch.randn(y.shape, generator=torch.Generator(device=dev).manual_seed(9), device=dev).to(dtype)
        y.backward(g)
        outs.append((y, x.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var))
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(4, 14, 14, 256), (3, 14, 14, 24), (2, 5, 3, 6)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_mask_equals_recomputed_mask(dev, shape, dtype, monkeypatch):
    """residual + ReLU BatchNorm: the backward reading the forward's ReLU bit mask (default) is
    bitwise equal to recomputing the mask from x and the residual (CS_BN_MASK=0), for V = 8 / 4 / 1"""
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import bn_act_nhwc
    torch.manual_seed(5)
    x0 = torch.randn(shape, device=dev).to(dtype)
    r0 = torch.randn(shape, device=dev).to(dtype)
    g = torch.randn(shape, device=dev).to(dtype)
    outs = []
    for m in ("0", "1"):
        monkeypatch.setenv("CS_BN_MASK", m)
        bn = nn.BatchNorm2d(shape[3]).to(dev)
        x, r = x0.clone().requires_grad_(), r0.clone().requires_grad_()
        y = bn_act_nhwc(bn, x, True, r)
        y.backward(g)
        outs.append((y, x.grad, r.grad, bn.weight.grad, bn.bias.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(2, 112, 112, 64), (3, 7, 9, 5), (1, 2, 3, 8)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_max_pool_nhwc_matches_torch(dev, shape, dtype):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn_nhwc import max_pool3s2_nhwc
    torch.manual_seed(1)
    x = torch.randn(shape, device=dev).to(dtype).requires_grad_()
    y = max_pool3s2_nhwc(x)
    xr = nchw(x.detach()).contiguous().requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(nchw(y), yr)
    g = torch.randn(yr.shape, device=dev).to(dtype)
    y.backward(nhwc(g))
    yr.backward(g)
    torch.testing.assert_close(nchw(x.grad).float(), xr.grad.float(), rtol=1e-2 if dtype == torch.bfloat16 else 1e-6,
                               atol=1e-2 if dtype == torch.bfloat16 else 1e-6)


def _step(model, x):
    model.zero_grad(set_to_none=True)
    y = model(x)
    y.square().mean().backward()
    return y.detach().clone(), [p.grad.clone() for p in model.parameters()]


def test_resnet18_nhwc_matches_nchw_module_path(dev):
    """a whole ResNet-18 forward/backward on the channels-last kernels == MIOpen + nn.BatchNorm2d (fp32),
    and bitwise equal to itself on a re-run"""
    from cs744_pytorch_distributed_tutorial_amd.models.resnet import resnet18
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn
    torch.manual_seed(0)
    a = resnet18(num_classes=10, layout="nhwc").to(dev)
    b = resnet18(num_classes=10, layout="nchw").to(dev)
    b.load_state_dict(a.state_dict())
    a2 = resnet18(num_classes=10, layout="nhwc").to(dev)
    a2.load_state_dict(a.state_dict())
    x = torch.randn(4, 3, 64, 64, device=dev)
    ya, ga = _step(a, x)
    ya2, ga2 = _step(a2, x)
    assert torch.equal(ya, ya2) and all(torch.equal(p, q) for p, q in zip(ga, ga2))
    orig = cnn.native_ok
    cnn.native_ok = lambda *args: False
    try:
        yb, gb = _step(b, x)
    finally:
        cnn.native_ok = orig
    torch.testing.assert_close(ya, yb, rtol=2e-3, atol=2e-3)
    for (n, _), pa, pb in zip(a.named_parameters(), ga, gb):
        torch.testing.assert_close(pa, pb, rtol=2e-2, atol=2e-3, msg=n)
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(ba.double(), bb.double(), rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bottleneck_residual_grad_sink_matches_autograd_sum(dev, dtype, monkeypatch):
    """bottlenecks (a downsampling one, two identity ones): the shortcut branch's gradient w.r.t.
    the block input taken into conv1's data-gradient GEMM
    (ResidualGradSink, default) == autograd summing it (CS_RES_SINK=0), input and every parameter
    gradient; and the sink really feeds the GEMM (its box is drained)"""
    from cs744_pytorch_distributed_tutorial_amd.models import resnet as rn
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc
    torch.manual_seed(6)
    down = nn.Sequential(rn.conv1x1(128, 256, 2), nn.BatchNorm2d(256))
    layer = nn.Sequential(rn.Bottleneck(128, 64, 2, down), rn.Bottleneck(256, 64), rn.Bottleneck(256, 64)).to(dev)
    x0 = torch.randn(4, 28, 28, 128, device=dev).to(dtype)
    g = torch.randn(4, 14, 14, 256, device=dev).to(dtype)
    boxes = []
    orig = cnn_nhwc.ResidualGradSink.apply

    def spy(x, box):
        boxes.append(box)
        return orig(x, box)

    monkeypatch.setattr(rn.ResidualGradSink, "apply", spy)
    outs = []
    for m in ("0", "1"):
        monkeypatch.setenv("CS_RES_SINK", m)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_()
        y = x
        for blk in layer:
            y = blk.forward_nhwc(y)
        y.backward(g)
        outs.append([x.grad.float()] + [p.grad.float() for p in layer.parameters()])
    assert len(boxes) == 3 and all(b.get("fused") and "g" not in b for b in boxes)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    for a, b in zip(*outs):
        assert ((a - b).norm() / (b.norm() + 1e-30)).item() < tol


def test_resnet50_nhwc_bf16_as_accurate_as_miopen_bf16(dev):
    """ResNet-50 under bf16 autocast, channels-last kernels vs MIOpen + the NCHW module path, both
    measured against the fp32 NCHW step on the same weights and batch: the native path's logit error
    and per-parameter gradient alignment are no worse than MIOpen's bf16 (bf16 error compounds over
    50 layers, so the two bf16 paths are compared through the fp32 reference, not to each other)"""
    from cs744_pytorch_distributed_tutorial_amd.models.resnet import resnet50
    torch.manual_seed(0)
    nets = {k: resnet50(num_classes=10, layout=k.split("_")[0]).to(dev) for k in ("nhwc_bf16", "nchw_bf16", "nchw_fp32")}
    sd = nets["nhwc_bf16"].state_dict()
    for m in nets.values():
        m.load_state_dict(sd)
    x = torch.randn(8, 3, 64, 64, device=dev)
    t = torch.randint(0, 10, (8,), device=dev)
    out = {}
    for k, m in nets.items():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=k.endswith("bf16")):
            y = m(x).float()
            loss = F.cross_entropy(y, t)
        loss.backward()
        out[k] = (y.detach().double(), [p.grad.double().flatten() for p in m.parameters()])
    yref, gref = out["nchw_fp32"]

    def err(k):
        y, g = out[k]
        cos = [float(a @ b / (a.norm() * b.norm())) for a, b in zip(g, gref) if b.norm() > 1e-6]
        return float((y - yref).norm() / yref.norm()), sum(cos) / len(cos), min(cos)

    e_nat, e_mio = err("nhwc_bf16"), err("nchw_bf16")
    assert e_nat[0] <= 2 * e_mio[0] + 0.02, (e_nat, e_mio)
    assert e_nat[1] >= e_mio[1] - 0.02 and e_nat[2] >= e_mio[2] - 0.1, (e_nat, e_mio)


def test_im2col_col2im_past_32bit_items(dev):
    """the gathers index work items in 32 bits; tensors past 2^31 items run in batch
    chunks instead of failing (the 224-px stem im2col crosses it near B = 850). 7300 images of
    64x64x8 bf16 through a 3x3 im2col = 2.15e9 column elements; images on both sides of every
    chunk boundary and the last one are checked against F.unfold, and col2im of the same columns
    against the adjoint on those images."""
    import torch.nn.functional as F
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C_ = native.C()
    B, H, C, Kp = 7300, 64, 8, 72
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, H, H, C, device=dev, generator=g).bfloat16()
    col = C_.im2col_nhwc(x, 3, 3, 1, 1, Kp)
    per = H * H * Kp
    assert col.numel() == B * per and col.numel() > 2 ** 31
    chunk = (2 ** 31 - 1) // per
    for b in sorted({0, chunk - 1, chunk, min(2 * chunk, B - 1), B - 1}):
        ref = F.unfold(x[b:b + 1].permute(0, 3, 1, 2).float(), 3, padding=1)  # [1, C*9 (c, r, s), HW]
        ref = ref.view(C, 9, H * H).permute(2, 1, 0).reshape(H * H, 9 * C)  # columns (r, s, c)
        got = col[b * H * H:(b + 1) * H * H, :9 * C].float()
        assert torch.equal(got, ref), b
    dx = C_.col2im_nhwc(col, B, H, H, C, 3, 3, 1, 1)
    for b in sorted({0, chunk, B - 1}):
        cb = col[b * H * H:(b + 1) * H * H, :9 * C].float().view(H * H, 9, C).permute(2, 1, 0).reshape(1, 9 * C, H * H)
        ref = F.fold(cb, (H, H), 3, padding=1).permute(0, 2, 3, 1)[0]
        torch.testing.assert_close(dx[b].float(), ref, rtol=1e-2, atol=1e-2)
    del col, dx
    torch.cuda.empty_cache()
