"""bf16 matrix-core GEMM (csrc/kernels/gemm_bf16.hip via C.mm_bf16(a, b) = a @ b) vs a plain
PyTorch reference of the same bf16 operands in fp64 (MI355X only). bf16 x bf16 products are exact
in fp32, so the fp32 output differs from the reference only by summation order; the bf16 output
by one rounding on top. All four operand layouts: a K-major ([M][K]) or M-major (a view of a
[K][M] tensor), b K-major (a view of [N][K], the nn.Linear weight) or N-major ([K][N])."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    return native.C()


def _ref(a, b):
    return a.double() @ b.double()


def _operands(M, N, K, layout, g, scale=1.0, uniform=True):
    """a [M, K], b [K, N] as views with the requested storage: layout = (a K-major, b K-major)"""
    def rnd(*shape):
        x = torch.rand(*shape, device="cuda", generator=g) * 2 - 1 if uniform else \
            torch.randn(*shape, device="cuda", generator=g)
        return (x * scale).bfloat16()
    ak, bk = layout
    p8 = lambda n: (n + 7) // 8 * 8  # noqa: E731  (row strides stay 16-byte multiples)
    a = rnd(M, K) if ak else rnd(K, p8(M))[:, :M].t()
    b = rnd(N, K).t() if bk else rnd(K, p8(N))[:, :N]
    return a, b


LAYOUTS = [(True, True), (True, False), (False, True), (False, False)]
LID = ["nt", "nn", "tt", "tn"]


SHAPES = [
    (256, 256, 64),      # one tile, one K-tile
    (512, 768, 4096),    # full tiles, long K
    (300, 260, 72),      # partial row / column tiles, partial last K-tile
    (1000, 1028, 136),   # N % 256 = 4, K % 64 = 8
    (64, 2048, 512),     # fewer rows than a tile
    (2304, 1024, 1024),  # grid not a multiple of 8 tiles (9 x 4 = 36 workgroups)
]


@pytest.mark.parametrize("layout", LAYOUTS, ids=LID)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_fp32_out(C, M, N, K, layout):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    a, b = _operands(M, N, K, layout, g)
    c = C.mm_bf16(a, b, True)
    ref = _ref(a, b)
    assert c.dtype == torch.float32 and c.shape == (M, N)
    err = (c.double() - ref).abs().max().item()
    # fp32 accumulation error bound ~ K * eps32 * sum|a b| (|a b| <= 1)
    assert err <= 1e-6 * K + 1e-5, err


@pytest.mark.parametrize("layout", LAYOUTS, ids=LID)
@pytest.mark.parametrize("M,N,K", SHAPES[:4])
def test_gemm_bf16_out(C, M, N, K, layout):
    g = torch.Generator(device="cuda").manual_seed(3 + M + N * 5 + K)
    a, b = _operands(M, N, K, layout, g, uniform=False)
    c = C.mm_bf16(a, b)
    assert c.dtype == torch.bfloat16
    ref = _ref(a, b)
    # one bf16 rounding of the fp32 result: relative 2^-8 of |C| plus the fp32 summation slack
    bound = ref.abs() * 2.0 ** -8 + 1e-5 * K
    assert bool(((c.double() - ref).abs() <= bound).all())


@pytest.mark.parametrize("layout", LAYOUTS, ids=LID)
def test_gemm_identity_asymmetric(C, layout):
    """A = I with an asymmetric B: C must be B exactly (catches a row/column-swapped store or a
    k-order slip in the transposed reads)."""
    K = 256
    ak, bk = layout
    eye = torch.eye(K, device="cuda").bfloat16()
    a = eye if ak else eye.t().contiguous().t()
    bm = (torch.arange(K * 384, device="cuda").reshape(K, 384) % 251 - 125).bfloat16()  # [K, N]
    b = bm.t().contiguous().t() if bk else bm
    c = C.mm_bf16(a, b, True)
    assert torch.equal(c, bm.float())


def test_gemm_accumulate_and_strided(C):
    torch.manual_seed(1)
    big = torch.randn(512, 640, device="cuda").bfloat16()
    a = big[:, 64:640]  # row stride 640, K = 576
    b = torch.randn(384, 576, device="cuda").bfloat16().t()
    acc = torch.randn(512, 384, device="cuda")
    acc0 = acc.clone()
    out = C.mm_bf16(a, b, acc=acc)
    assert out.data_ptr() == acc.data_ptr()
    ref = acc0.double() + _ref(a, b)
    assert (acc.double() - ref).abs().max().item() < 1e-3


def test_gemm_linear_layer_products(C):
    """the three GEMMs of a linear layer on one weight, as ops/lm.py issues them"""
    torch.manual_seed(2)
    x = torch.randn(1024, 768, device="cuda").bfloat16()
    w = (torch.randn(1280, 768, device="cuda") * 0.05).bfloat16()
    dy = torch.randn(1024, 1280, device="cuda").bfloat16()
    y = C.mm_bf16(x, w.t(), True)
    dx = C.mm_bf16(dy, w, True)
    dw = C.mm_bf16(dy.t(), x, True)
    for got, ref in ((y, x.double() @ w.double().t()), (dx, dy.double() @ w.double()),
                     (dw, dy.double().t() @ x.double())):
        assert (got.double() - ref).abs().max().item() < 1e-6 * ref.abs().max().item() * 64


def test_gemm_rejects_unsupported(C):
    a = torch.randn(64, 12, device="cuda").bfloat16()  # K-major with K % 8 != 0
    b = torch.randn(12, 64, device="cuda").bfloat16()
    with pytest.raises(RuntimeError):
        C.mm_bf16(a, b.t().contiguous().t())
    with pytest.raises(RuntimeError):
        C.mm_bf16(a.float(), b.float())
    with pytest.raises(RuntimeError):
        C.mm_bf16(torch.randn(64, 64, 2, device="cuda").bfloat16()[:, :, 0], b[:, :64].contiguous())


@pytest.mark.parametrize("layout", [(True, True), (False, False)], ids=["nt", "tn"])
def test_gemm_split_k(C, layout):
    """reduction split over slabs (the weight-gradient shape: small output, long K), summed in
    fixed order; also into an accumulator"""
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 256, 512, 8200
    a, b = _operands(M, N, K, layout, g)
    ref = _ref(a, b)
    one = C.mm_bf16(a, b, True, splits=1)
    auto = C.mm_bf16(a, b, True)
    three = C.mm_bf16(a, b, True, splits=3)
    for c in (one, auto, three):
        assert (c.double() - ref).abs().max().item() <= 1e-6 * K + 1e-5
    assert torch.equal(auto, C.mm_bf16(a, b, True))  # deterministic
    acc = torch.ones(M, N, device="cuda")
    C.mm_bf16(a, b, acc=acc, splits=4)
    assert (acc.double() - (ref + 1)).abs().max().item() <= 1e-6 * K + 1e-5


# (B, Cin, H, W, Cout, k, stride, pad): ResNet-50 bf16 GEMM convolutions (1x1, strided 1x1 through
# im2col, a deep 3x3 through im2col) on the native GEMM (CS_CONV_GEMM=native) vs fp64
@pytest.mark.parametrize("geo", [(2, 64, 14, 14, 256, 1, 1, 0), (2, 256, 14, 14, 64, 1, 1, 0),
                                 (2, 256, 14, 14, 512, 1, 2, 0), (2, 256, 7, 7, 256, 3, 1, 1)])
def test_conv_nhwc_on_native_gemm(C, geo, monkeypatch):
    import torch.nn as nn
    import torch.nn.functional as F
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc
    monkeypatch.setattr(cnn_nhwc, "_CONV_GEMM", "native")
    B, Ci, H, W, Co, k, st, pad = geo
    torch.manual_seed(sum(geo))
    conv = nn.Conv2d(Ci, Co, k, stride=st, padding=pad, bias=False).cuda()
    x = torch.randn(B, Ci, H, W, device="cuda").bfloat16()
    xh = x.permute(0, 2, 3, 1).contiguous().requires_grad_()
    y = cnn_nhwc.conv_nhwc(xh, conv)
    xr = x.double().requires_grad_()
    wr = conv.weight.detach().bfloat16().double().requires_grad_()
    yr = F.conv2d(xr, wr, None, st, pad)
    torch.testing.assert_close(y.permute(0, 3, 1, 2).double(), yr, rtol=1e-2, atol=1e-2)
    g = torch.randn(yr.shape, device="cuda").bfloat16()
    y.backward(g.permute(0, 2, 3, 1).contiguous())
    yr.backward(g.double())
    torch.testing.assert_close(xh.grad.permute(0, 3, 1, 2).double(), xr.grad, rtol=1e-2, atol=1e-2)
    # the weight gradient leaves the GEMM in fp32 (bf16 operands): only summation order differs
    torch.testing.assert_close(conv.weight.grad.double(), wr.grad, rtol=1e-4, atol=1e-3)


def test_gemm_bn_stats_epilogue(C):
    """per-256-row-tile (mean, M2) of the bf16 output, from the GEMM epilogue, vs fp64 of y itself"""
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 700, 384, 320  # a partial last row tile
    a = (torch.randn(M, K, device="cuda", generator=g) + 0.3).bfloat16()
    b = torch.randn(N, K, device="cuda", generator=g).bfloat16().t()
    y, tiles = C.mm_bf16_bn_stats(a, b)
    assert torch.equal(y, C.mm_bf16(a, b))
    assert tiles.shape == (3, N, 2)
    yd = y.double()
    for t in range(3):
        blk = yd[256 * t:256 * (t + 1)]
        mean = blk.mean(0)
        m2 = ((blk - mean) ** 2).sum(0)
        torch.testing.assert_close(tiles[t, :, 0].double(), mean, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(tiles[t, :, 1].double(), m2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_bn_nhwc_from_gemm_tiles_matches_stats_pass(C, relu, residual):
    g = torch.Generator(device="cuda").manual_seed(6)
    B, H, W, K, Co = 4, 15, 13, 256, 256
    M = B * H * W
    a = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(Co, K, device="cuda", generator=g) * 0.1).bfloat16()
    y, tiles = C.mm_bf16_bn_stats(a, w.t())
    x = y.view(B, H, W, Co)
    res = torch.randn(B, H, W, Co, device="cuda", generator=g).bfloat16() if residual else None
    gam = torch.rand(Co, device="cuda", generator=g) + 0.5
    bet = torch.randn(Co, device="cuda", generator=g)
    outs = []
    for t in (None, tiles):
        rm, rv = torch.zeros(Co, device="cuda"), torch.ones(Co, device="cuda")
        nbt = torch.zeros((), dtype=torch.long, device="cuda")
        yo, stat, _ = C.bn_nhwc_fwd(x, res, gam, bet, rm, rv, nbt, 0.1, 1e-5, relu, False, t)
        outs.append((yo, stat, rm, rv, nbt))
    (y0, s0, rm0, rv0, n0), (y1, s1, rm1, rv1, n1) = outs
    torch.testing.assert_close(s1, s0, rtol=2e-5, atol=2e-5)
    torch.testing.assert_close(rm1, rm0, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(rv1, rv0, rtol=2e-5, atol=2e-6)
    assert int(n0) == int(n1) == 1
    # same scale/shift up to float rounding -> outputs within a bf16 ulp
    torch.testing.assert_close(y1.float(), y0.float(), rtol=1e-2, atol=1e-2)


def test_resnet_bottleneck_native_gemm_close_to_blas(C, monkeypatch):
    """a ResNet-50 bottleneck step (bf16 autocast, channels-last) with its GEMM convolutions and
    the BatchNorm statistics on the native GEMM vs hipBLASLt + the statistics pass"""
    from cs744_pytorch_distributed_tutorial_amd.models import resnet as rn
    from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc
    torch.manual_seed(8)
    # 1024 -> 256 -> 1024 channels: every GEMM of the block is >= 256 wide (the "wgrad" mode's bar)
    blk0 = rn.Bottleneck(1024, 256).cuda()
    x0 = torch.randn(8, 14, 14, 1024, device="cuda").bfloat16()
    res = {}
    for mode in ("blas", "native", "wgrad"):
        monkeypatch.setattr(cnn_nhwc, "_CONV_GEMM", mode)
        blk = rn.Bottleneck(1024, 256).cuda()
        blk.load_state_dict(blk0.state_dict())
        x = x0.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = blk.forward_nhwc(x)
        y.float().square().mean().backward()
        res[mode] = (y.float(), x.grad.float(), blk.conv1.weight.grad, blk.bn3.running_var.clone())
    for a, b in zip(res["native"], res["blas"]):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2)
    # weight gradients only: the forward is hipBLASLt's, bit for bit
    assert torch.equal(res["wgrad"][0], res["blas"][0])
    for a, b in zip(res["wgrad"][1:], res["blas"][1:]):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2)
