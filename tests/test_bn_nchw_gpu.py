"""Fused training BatchNorm2d (+residual) (+ReLU) on NCHW (csrc/kernels/bn_nchw.hip) vs the
PyTorch ops it replaces (F.batch_norm in training mode, add, relu) in fp32/fp64: outputs,
running statistics and every gradient; plus a ResNet forward/backward against the module path."""
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


def _ref(bn, x, relu, res):
    y = F.batch_norm(x.double(), bn.running_mean.double(), bn.running_var.double(), bn.weight.double(),
                     bn.bias.double(), True, bn.momentum, bn.eps)
    if res is not None:
        y = y + res.double()
    return F.relu(y) if relu else y


SHAPES = [(4, 64, 56, 56), (8, 32, 7, 7), (3, 16, 14, 14), (2, 8, 5, 3)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_bn_act_matches_torch(dev, shape, dtype, relu, residual):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn import bn_act, native_ok
    torch.manual_seed(hash((shape, relu, residual)) % 1000)
    C = shape[1]
    bn = nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
    ref_bn = nn.BatchNorm2d(C).to(dev)
    ref_bn.load_state_dict(bn.state_dict())
    x = (torch.randn(shape, device=dev) * 2 + 0.7).to(dtype).requires_grad_()
    res = (torch.randn(shape, device=dev)).to(dtype).requires_grad_() if residual else None
    assert native_ok(bn, x, res)
    y = bn_act(bn, x, relu, res)
    xr = x.detach().double().requires_grad_()
    rr = res.detach().double().requires_grad_() if residual else None
    wr = ref_bn.weight.detach().double().requires_grad_()
    br = ref_bn.bias.detach().double().requires_grad_()
    yr = F.batch_norm(xr, ref_bn.running_mean.double(), ref_bn.running_var.double(), wr, br, True, 0.1, 1e-5)
    if residual:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.double(), yr, **tol)
    # running statistics (momentum 0.1, unbiased variance)
    M = shape[0] * shape[2] * shape[3]
    xd = x.detach().double()
    mean = xd.mean((0, 2, 3))
    var = xd.var((0, 2, 3), unbiased=True) if M > 1 else xd.var((0, 2, 3), unbiased=False)
    rm0 = ref_bn.running_mean.double()
    torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0 + 0.1 * mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), 0.9 * 1.0 + 0.1 * var, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == 1
    # gradients
    g = torch.randn(shape, device=dev).to(dtype)
    y.backward(g)
    yr.backward(g.double())
    gt = dict(rtol=1e-3, atol=1e-3) if dtype == torch.float32 else dict(rtol=5e-2, atol=5e-2)
    torch.testing.assert_close(x.grad.double(), xr.grad, **gt)
    torch.testing.assert_close(bn.weight.grad.double(), wr.grad, rtol=1e-3, atol=1e-2 if dtype == torch.bfloat16 else 1e-3)
    torch.testing.assert_close(bn.bias.grad.double(), br.grad, rtol=1e-3, atol=1e-2 if dtype == torch.bfloat16 else 1e-3)
    if residual:
        torch.testing.assert_close(res.grad.double(), rr.grad, **gt)


def test_resnet_native_bn_matches_module_path(dev, monkeypatch):
    """ResNet-18 forward/backward with the fused kernels == the nn.BatchNorm2d/relu/add path (fp32)."""
    from cs744_pytorch_distributed_tutorial_amd.models.resnet import resnet18
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn
    torch.manual_seed(0)
    a = resnet18(num_classes=10, layout="nchw").to(dev)
    b = resnet18(num_classes=10, layout="nchw").to(dev)
    b.load_state_dict(a.state_dict())
    x = torch.randn(4, 3, 64, 64, device=dev)
    ya = a(x)
    ya.square().mean().backward()
    monkeypatch.setattr(cnn, "native_ok", lambda *args: False)
    yb = b(x)
    yb.square().mean().backward()
    torch.testing.assert_close(ya, yb, rtol=2e-3, atol=2e-3)
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=2e-2, atol=2e-3, msg=n)
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        torch.testing.assert_close(ba.double(), bb.double(), rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("shape", [(2, 3, 112, 112), (3, 5, 7, 9), (1, 2, 2, 3)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_max_pool3s2_matches_torch(dev, shape, dtype):
    from cs744_pytorch_distributed_tutorial_amd.ops.cnn import max_pool3s2
    torch.manual_seed(1)
    x = torch.randn(shape, device=dev).to(dtype).requires_grad_()
    y = max_pool3s2(x)
    xr = x.detach().clone().requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y, yr)
    g = torch.randn(y.shape, device=dev).to(dtype)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad.float(), xr.grad.float(), rtol=1e-2 if dtype == torch.bfloat16 else 1e-6,
                               atol=1e-2 if dtype == torch.bfloat16 else 1e-6)
