"""bf16 NHWC implicit-GEMM convolution (csrc/kernels/conv_nhwc.hip) vs a float64 reference of the
same op on the same bf16-rounded operands: forward, data gradient and weight gradient for 3x3 /
1x1 / 7x7 kernels, strides 1 and 2, channel counts that do and do not fill a 128-wide tile, and
the ResNet layer through ops/cnn_nhwc.py (implicit path vs the im2col + GEMM path)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    return native.C()


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


SHAPES = [  # B, H, W, C, Co, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 64, 128, 3, 2, 1),
    (3, 7, 9, 96, 160, 3, 1, 1),
    (2, 16, 16, 128, 64, 1, 2, 0),
    (2, 8, 8, 256, 256, 1, 1, 0),
    (1, 15, 15, 32, 96, 7, 2, 3),
    (4, 5, 5, 512, 512, 3, 1, 1),
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_nhwc_bf16_matches_fp64(C, shape):
    B, H, W, Ci, Co, R, st, pad = shape
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    x = torch.randn(B, H, W, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, R, Ci, device=dev) / (R * R * Ci) ** 0.5).to(torch.bfloat16)
    # float64 reference on the bf16 values
    xr = x.double().cpu().permute(0, 3, 1, 2).requires_grad_()
    wr = w.double().cpu().permute(0, 3, 1, 2).requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pad)
    Ho, Wo = yr.shape[2], yr.shape[3]
    y = C.conv_nhwc_bf16(0, x, w, R, R, st, pad, 0, 0)
    torch.cuda.synchronize()
    assert y.shape == (B, Ho, Wo, Co)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 5e-3
    dy = torch.randn(B, Ho, Wo, Co, device=dev).to(torch.bfloat16)
    yr.backward(dy.double().cpu().permute(0, 3, 1, 2))
    dx = C.conv_nhwc_bf16(1, dy, w.permute(3, 1, 2, 0).contiguous(), R, R, st, pad, H, W)
    dw = C.conv_nhwc_bf16(2, dy, x, R, R, st, pad, 0, 0)
    torch.cuda.synchronize()
    assert dx.shape == x.shape and dw.shape == (Co, R * R * Ci) and dw.dtype == torch.float32
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 5e-3
    # fp32 accumulation of exact bf16 products: only the summation order differs
    assert _rel(dw.view(Co, R, R, Ci).permute(0, 3, 1, 2), wr.grad) < 1e-4


def test_conv_nhwc_bf16_deterministic(C):
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    x = torch.randn(8, 28, 28, 128, device=dev).to(torch.bfloat16)
    dy = torch.randn(8, 28, 28, 128, device=dev).to(torch.bfloat16)
    a = C.conv_nhwc_bf16(2, dy, x, 3, 3, 1, 1, 0, 0)
    b = C.conv_nhwc_bf16(2, dy, x, 3, 3, 1, 1, 0, 0)
    assert torch.equal(a, b)


def test_conv_nhwc_rejects_bad_shapes(C):
    dev = torch.device("cuda", 0)
    x = torch.randn(1, 8, 8, 4, device=dev).to(torch.bfloat16)  # C = 4: not a multiple of 32
    w = torch.randn(64, 3, 3, 4, device=dev).to(torch.bfloat16)
    with pytest.raises(RuntimeError):
        C.conv_nhwc_bf16(0, x, w, 3, 3, 1, 1, 0, 0)


@pytest.mark.parametrize("stride,k", [(1, 3), (2, 3), (2, 1)])
def test_resnet_conv_layer_implicit_vs_im2col(C, stride, k, monkeypatch):
    """ops/cnn_nhwc.conv_nhwc under bf16 autocast: the implicit-GEMM path (CS_CONV_IMPLICIT=2: every
    conv it serves) and the im2col + GEMM path (=0) agree on y, dx and dW to bf16 rounding."""
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc
    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    conv = torch.nn.Conv2d(64, 128, k, stride, k // 2, bias=False).to(dev)
    x0 = torch.randn(4, 16, 16, 64, device=dev).to(torch.bfloat16)
    g0 = torch.randn(4, 16 // stride, 16 // stride, 128, device=dev).to(torch.bfloat16)
    outs = []
    for mode in ("0", "2"):
        monkeypatch.setenv("CS_CONV_IMPLICIT", mode)
        x = x0.clone().requires_grad_()
        conv.weight.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = cnn_nhwc.conv_nhwc(x, conv)
        assert y.shape == g0.shape
        y.backward(g0)
        outs.append((y.detach().float(), x.grad.float(), conv.weight.grad.float()))
    for a, b in zip(*outs):
        assert _rel(a, b) < 1e-2


@pytest.mark.parametrize("shape", [(2, 30, 30, 64, 7, 2, 3), (1, 17, 19, 32, 3, 1, 1), (2, 224, 224, 64, 7, 2, 3)],
                         ids=lambda s: "x".join(map(str, s)))
def test_conv_nhwc_stem_c4_matches_fp64(C, shape):
    """C4 mode (the 4-channel stem): kernel rows padded to 8 taps, forward and weight gradient vs f64"""
    B, H, W, Co, R, st, pad = shape
    torch.manual_seed(3)
    dev = torch.device("cuda", 0)
    x = torch.randn(B, H, W, 4, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, R, R, 4, device=dev) / (R * R * 4) ** 0.5).to(torch.bfloat16)
    wp = torch.nn.functional.pad(w, (0, 0, 0, 8 - R)).contiguous()  # [Co, R, 8, 4], zero taps s >= R
    xr = x.double().cpu().permute(0, 3, 1, 2)
    wr = w.double().cpu().permute(0, 3, 1, 2).requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pad)
    y = C.conv_nhwc_bf16(0, x, wp, R, R, st, pad, 0, 0)
    torch.cuda.synchronize()
    assert y.shape == (B, yr.shape[2], yr.shape[3], Co)
    assert _rel(y.permute(0, 3, 1, 2), yr) < 5e-3
    dy = torch.randn(*y.shape, device=dev).to(torch.bfloat16)
    yr.backward(dy.double().cpu().permute(0, 3, 1, 2))
    dw = C.conv_nhwc_bf16(2, dy, x, R, R, st, pad, 0, 0)
    torch.cuda.synchronize()
    assert dw.shape == (Co, R * 32)
    assert _rel(dw.view(Co, R, 8, 4)[:, :, :R].permute(0, 3, 1, 2), wr.grad) < 1e-4


def test_resnet_stem_implicit_vs_im2col(C, monkeypatch):
    """the ResNet stem (3 -> 64, 7x7/2, image padded to 4 channels) through ops/cnn_nhwc.conv_nhwc:
    C4 implicit path (default) vs im2col + GEMM (CS_CONV_IMPLICIT=0), y and dW"""
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc
    dev = torch.device("cuda", 0)
    torch.manual_seed(4)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
    x = cnn_nhwc.to_nhwc(torch.randn(4, 3, 64, 64, device=dev), torch.bfloat16, pad_c=1)
    g0 = torch.randn(4, 32, 32, 64, device=dev).to(torch.bfloat16)
    outs = []
    for mode in ("0", "1"):
        monkeypatch.setenv("CS_CONV_IMPLICIT", mode)
        conv.weight.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = cnn_nhwc.conv_nhwc(x, conv)
        y.backward(g0)
        outs.append((y.detach().float(), conv.weight.grad.float()))
    for a, b in zip(*outs):
        assert _rel(a, b) < 1e-2


@pytest.mark.parametrize("S,shape", [(64, (64, 256)), (3, (5, 12)), (512, (64, 224)), (1, (8, 8))])
def test_slab_sum_matches_fp64_and_is_deterministic(C, S, shape):
    dev = torch.device("cuda", 0)
    torch.manual_seed(12)
    part = torch.randn(S, *shape, device=dev)
    a = C.slab_sum(part)
    b = C.slab_sum(part)
    torch.cuda.synchronize()
    assert a.shape == shape and torch.equal(a, b)
    assert _rel(a, part.double().sum(0)) < 1e-6
