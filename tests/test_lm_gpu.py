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
def test_swiglu(dev, dtype):
    from cs744_pytorch_distributed_tutorial_amd.ops import lm
    a = torch.randn(3, 17, 352, device=dev).to(dtype).requires_grad_()
    b = torch.randn(3, 17, 352, device=dev).to(dtype).requires_grad_()
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
