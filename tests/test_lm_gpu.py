"""Decoder-LM gfx950 kernels (RMSNorm, SwiGLU, RoPE; fp32 + bf16) vs plain
PyTorch fp32 references, forward and backward; ResNet-50 / Llama-tiny steps
through the autograd-path trainer (MI355X only)."""
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


TOL = {torch.float32: dict(rtol=1e-5, atol=1e-5), torch.bfloat16: dict(rtol=2e-2, atol=2e-2)}


def _ref_grads(fn, inputs, gy):
    ins = [t.detach().float().requires_grad_() for t in inputs]
    out = fn(*ins)
    out.backward(gy.float())
    return out.detach(), [t.grad for t in ins]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(4, 7, 256), (3, 4096), (2, 5, 1000)])
def test_rmsnorm(dev, dtype, shape):
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    torch.manual_seed(0)
    x = torch.randn(*shape, device=dev).to(dtype).requires_grad_()
    w = (torch.rand(shape[-1], device=dev) + 0.5).requires_grad_()
    y = lm.rms_norm(x, w, 1e-5)
    gy = torch.randn_like(y)
    y.backward(gy)
    ry, (rgx, rgw) = _ref_grads(lambda a, b: lm.rms_norm_ref(a, b, 1e-5), [x, w], gy)
    torch.testing.assert_close(y.float(), ry, **TOL[dtype])
    torch.testing.assert_close(x.grad.float(), rgx, **TOL[dtype])
    torch.testing.assert_close(w.grad.float(), rgw, rtol=2e-2 if dtype == torch.bfloat16 else 1e-4,
                               atol=5e-2 if dtype == torch.bfloat16 else 1e-4)


@pytest.mark.parametrize("shape", [(2, 9, 4096), (3, 1000), (5, 8192)])
def test_rmsnorm_fp32_stream_bf16_out(dev, shape):
    """under bf16 autocast: fp32 residual stream in, bf16 normalised activations out (no cast pass),
    bf16 incoming gradient, fp32 dx and weight gradient"""
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    torch.manual_seed(1)
    x = torch.randn(*shape, device=dev).requires_grad_()
    w = (torch.rand(shape[-1], device=dev) + 0.5).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lm.rms_norm(x, w, 1e-5)
    assert y.dtype == torch.bfloat16
    gy = torch.randn(shape, device=dev).bfloat16()
    y.backward(gy)
    assert x.grad.dtype == torch.float32 and w.grad.dtype == torch.float32
    ry, (rgx, rgw) = _ref_grads(lambda a, b: lm.rms_norm_ref(a, b, 1e-5), [x, w], gy.float())
    torch.testing.assert_close(y.float(), ry, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(x.grad, rgx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w.grad, rgw, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(3, 17, 352), (5, 7, 9)])  # 4-wide kernels / scalar kernels
def test_swiglu(dev, dtype, shape):
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    a = torch.randn(*shape, device=dev).to(dtype).requires_grad_()
    b = torch.randn(*shape, device=dev).to(dtype).requires_grad_()
    y = lm.swiglu(a, b)
    gy = torch.randn_like(y)
    y.backward(gy)
    ry, (ga, gb) = _ref_grads(lm.swiglu_ref, [a, b], gy)
    torch.testing.assert_close(y.float(), ry, **TOL[dtype])
    torch.testing.assert_close(a.grad.float(), ga, **TOL[dtype])
    torch.testing.assert_close(b.grad.float(), gb, **TOL[dtype])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rope(dev, dtype):
    from cs744_pytorch_distributed_tutorial_amd.models.llama import rope_tables
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    B, S, H, hd = 2, 33, 4, 64
    cos, sin = rope_tables(S, hd, 500000.0, dev)
    x = torch.randn(B, S, H, hd, device=dev).to(dtype).requires_grad_()
    y = lm.rope(x, cos, sin)
    gy = torch.randn_like(y)
    y.backward(gy)
    ry, (gx,) = _ref_grads(lambda t: lm.rope_ref(t, cos, sin), [x], gy)
    torch.testing.assert_close(y.float(), ry, **TOL[dtype])
    torch.testing.assert_close(x.grad.float(), gx, **TOL[dtype])


def test_llama_tiny_trains_bf16(dev):
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import TorchTrainer
    tr = TorchTrainer("llama-tiny", 8, dev, dtype="bf16", lr=0.05, weight_decay=0.0)
    losses = []
    for _ in range(30):
        tr.step()
        losses.append(tr.last_loss())
    assert all(v == v for v in losses)
    assert sum(losses[-5:]) / 5 < sum(losses[:3]) / 3


def test_resnet50_step(dev):
    from cs744_pytorch_distributed_tutorial_amd.runtime.torch_trainer import TorchTrainer
    tr = TorchTrainer("resnet50", 8, dev, dtype="bf16")
    tr.step()
    tr.step()
    assert tr.last_loss() == tr.last_loss()


def test_shadow_linear_matches_autocast_linear_and_sgd_keeps_shadow(dev):
    """ShadowLinear under bf16 autocast == nn.Linear under autocast (same bf16 GEMM), fp32 weight
    gradient at least as accurate; FusedSGD rewrites the bf16 shadow with the updated weight (bit-equal
    to a fresh cast), and an in-place weight change outside the optimizer invalidates it"""
    from cs744_pytorch_distributed_tutorial_amd.ops.lm import ShadowLinear
    from cs744_pytorch_distributed_tutorial_amd.ops.optim import FusedSGD
    torch.manual_seed(3)
    a = ShadowLinear(256, 384, bias=False).to(dev)
    b = torch.nn.Linear(256, 384, bias=False).to(dev)
    b.load_state_dict(a.state_dict())
    x = torch.randn(2, 64, 256, device=dev)
    gy = torch.randn(2, 64, 384, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya, yb = a(x), b(x)
    assert ya.dtype == yb.dtype == torch.bfloat16
    assert torch.equal(ya, yb)
    ya.backward(gy.bfloat16())
    yb.backward(gy.bfloat16())
    ref = gy.bfloat16().reshape(-1, 384).t().double() @ x.bfloat16().double().reshape(-1, 256)
    assert a.weight.grad.dtype == torch.float32
    err_a = (a.weight.grad.double() - ref).norm() / ref.norm()
    err_b = (b.weight.grad.double() - ref).norm() / ref.norm()
    assert err_a <= err_b + 1e-6 and err_a < 1e-5, (float(err_a), float(err_b))
    opt = FusedSGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    opt.step()
    sh = a.weight._cs_bf16_shadow
    assert torch.equal(sh, a.weight.detach().to(torch.bfloat16))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a(x)
    assert a.weight._cs_bf16_shadow is sh  # still valid: the fused pass kept it in step
    with torch.no_grad():
        a.weight.mul_(0.5)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a(x)
    assert torch.equal(a.weight._cs_bf16_shadow, a.weight.detach().to(torch.bfloat16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("R,V", [(64, 1024), (7, 128256), (33, 8)])
def test_cross_entropy_matches_torch(dev, dtype, R, V):
    from cs744_pytorch_distributed_tutorial_amd.ops.lm import cross_entropy
    torch.manual_seed(R)
    x = (torch.randn(R, V, device=dev) * 3).to(dtype).requires_grad_()
    t = torch.randint(0, V, (R,), device=dev)
    loss = cross_entropy(x, t)
    xr = x.detach().double().requires_grad_()
    ref = torch.nn.functional.cross_entropy(xr, t)
    torch.testing.assert_close(loss.double(), ref, rtol=1e-5, atol=1e-5)
    (2.5 * loss).backward()
    (2.5 * ref).backward()
    tol = dict(rtol=1e-4, atol=1e-6) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), xr.grad, **tol)


@pytest.mark.parametrize("out_features", [32001, 50257, 390])
def test_shadow_linear_odd_shapes_fall_back(dev, out_features):
    """Shapes the native GEMM cannot read in place (an odd vocabulary: N % 4 != 0 / ld % 8 != 0;
    an expanded stride-0 upstream gradient from y.sum().backward()) run through torch.mm instead
    of raising in backward; the fp32 weight gradient matches the fp64 product."""
    from cs744_pytorch_distributed_tutorial_amd.ops.lm import ShadowLinear, gemm_operands_ok
    torch.manual_seed(0)
    lin = ShadowLinear(264, out_features, bias=False).to(dev)
    x = torch.randn(24, 264, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lin(x)
    y.float().sum().backward()  # expanded (stride-0) upstream gradient
    ref = torch.ones(24, out_features, dtype=torch.float64, device=dev).t() @ x.to(torch.bfloat16).double()
    assert lin.weight.grad.dtype == torch.float32
    torch.testing.assert_close(lin.weight.grad.double(), ref, rtol=2e-2, atol=2e-1)
    g = torch.ones(1, 1, device=dev, dtype=torch.bfloat16).expand(24, out_features)
    assert not gemm_operands_ok(g.t(), x.to(torch.bfloat16))


def test_mm_bf16_empty_reduction_is_zero(dev):
    """K = 0 (an empty token batch's weight gradient) returns zeros like torch.mm, not uninitialised
    memory; an accumulator comes back unchanged."""
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    a = torch.empty(64, 0, device=dev, dtype=torch.bfloat16)
    b = torch.empty(0, 128, device=dev, dtype=torch.bfloat16)
    for out_f32 in (False, True):
        c = native.C().mm_bf16(a, b, out_f32)
        assert c.shape == (64, 128) and bool((c == 0).all())
    acc = torch.full((64, 128), 3.0, device=dev)
    assert torch.equal(native.C().mm_bf16(a, b, True, acc), torch.full_like(acc, 3.0))
