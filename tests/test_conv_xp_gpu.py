"""Numerics of the pre-split ("XP") conv GEMMs (csrc/kernels/conv_xp.hip): operands as three
bf16 planes from ``split3``, six-product split-bf16 MFMA maths — held to the same float64
tolerance as the f32 MFMA kernels (tests/test_conv_bn_gpu.py). MI355X only."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    native.C()
    return torch.device("cuda", 0)


def _close(a, b, rel=2e-5):
    a = a.double().cpu()
    b = b.double().cpu()
    scale = b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert err <= rel * scale, f"max err {err:.3e} vs scale {scale:.3e}"


# (B, H, cin, cout): VGG-11 layer shapes at small batches; (3, 2, ...) has a ragged wgrad K (12)
SHAPES = [(2, 16, 64, 128), (2, 8, 128, 256), (3, 4, 256, 512), (4, 2, 512, 512), (3, 2, 512, 512)]
# (bm, bn, bk, kg, nb) — every variant cs_conv_xp_ok admits (nb 0 = deepest ring that fits)
XP_TILES = [(64, 64, 32, 1, 0), (128, 64, 32, 1, 0), (64, 128, 32, 1, 0), (128, 128, 32, 1, 0), (64, 64, 64, 1, 0),
            (128, 64, 64, 1, 0), (64, 128, 64, 1, 0), (128, 128, 32, 2, 0), (64, 64, 64, 2, 0), (128, 64, 64, 2, 0),
            (64, 128, 64, 2, 0), (64, 64, 32, 1, 2), (64, 64, 32, 1, 3), (128, 64, 32, 1, 2), (64, 128, 32, 1, 2)]
SPLITS = [1, 3]


def _inputs(B, H, cin, cout, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    gy = torch.randn(B, cout, H, H, generator=g, dtype=torch.float64)
    return x, w, b, gy


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def test_xp_table_mirrors_kernel(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    got = [(bm, bn, bk, kg, nb) for bm in (64, 128) for bn in (64, 128) for bk in (16, 32, 64) for kg in (1, 2, 4)
           for nb in range(5) if C.conv_xp_ok(bm, bn, bk, kg, nb)]
    assert sorted(got) == sorted(XP_TILES)


def test_split3_exact(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    x = torch.randn(4096, device=dev) * torch.logspace(-20, 20, 4096, device=dev)
    p = Fn.split3(x).double()  # [n/8, 3, 8]
    h, m, lo = (p[:, i, :].reshape(-1) for i in range(3))
    rec = h + m + lo
    assert ((rec - x.double()).abs() <= 2.0 ** -26 * x.double().abs()).all()
    assert (h.float() == x.bfloat16().float()).all()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tile", XP_TILES)
@pytest.mark.parametrize("splits", SPLITS)
def test_xp_fwd_and_stats(dev, shape, tile, splits):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, bk, kg, nb = tile
    x, w, b, _ = _inputs(B, H, cin, cout)
    ref = F.conv2d(x, w, b, padding=1).permute(0, 2, 3, 1).reshape(-1, cout)
    x3 = Fn.split3(_nhwc(x).float().to(dev))
    w3 = Fn.split3(w.permute(0, 2, 3, 1).contiguous().float().to(dev))
    y, st, rows = Fn.conv_fwd_xp(x3, w3, b.float().to(dev), B, H, H, cin, cout, bm=bm, bn=bn, bk=bk, kg=kg,
                                 splits=splits, stats=True, nb=nb)
    _close(y, ref)
    M = ref.shape[0]
    for t in range(st.shape[0]):
        seg = ref[t * rows:min(M, (t + 1) * rows)]
        mu = seg.mean(0)
        _close(st[t, :, 0], mu, 1e-4)
        _close(st[t, :, 1], ((seg - mu) ** 2).sum(0), 1e-4)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tile", XP_TILES)
@pytest.mark.parametrize("splits", SPLITS)
def test_xp_dgrad(dev, shape, tile, splits):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, bk, kg, nb = tile
    x, w, _, gy = _inputs(B, H, cin, cout, 1)
    ref = torch.nn.grad.conv2d_input(x.shape, w, gy, padding=1).permute(0, 2, 3, 1).reshape(-1, cin)
    dz3 = Fn.split3(_nhwc(gy).float().to(dev))
    w3 = Fn.split3(w.permute(0, 2, 3, 1).contiguous().float().to(dev))
    dx = Fn.conv_dgrad_xp(dz3, w3, B, H, H, cin, cout, bm=bm, bn=bn, bk=bk, kg=kg, splits=splits, nb=nb)
    _close(dx, ref)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tile", XP_TILES)
@pytest.mark.parametrize("splits", SPLITS)
def test_xp_wgrad(dev, shape, tile, splits):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, bk, kg, nb = tile
    x, w, _, gy = _inputs(B, H, cin, cout, 2)
    ref = torch.nn.grad.conv2d_weight(x, w.shape, gy, padding=1).permute(0, 2, 3, 1)
    dz3 = Fn.split3(_nhwc(gy).float().to(dev))
    x3 = Fn.split3(_nhwc(x).float().to(dev))
    dw = Fn.conv_wgrad_xp(dz3, x3, B, H, H, cin, cout, bm=bm, bn=bn, bk=bk, kg=kg, splits=splits, nb=nb)
    _close(dw, ref)
