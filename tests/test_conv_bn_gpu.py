"""Numerics of the implicit-GEMM conv (fwd / dgrad / wgrad) and fused BN+ReLU(+pool)
kernels vs plain PyTorch fp32/fp64 references (MI355X only)."""
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


# (B, H, cin, cout) — VGG-11 layer shapes at a small batch, plus conv0 (padded cin 4)
SHAPES = [(2, 32, 3, 64), (2, 16, 64, 128), (2, 8, 128, 256), (3, 4, 256, 512), (4, 2, 512, 512)]
TILES = [(64, 64, 1, 16), (128, 64, 1, 16), (64, 128, 3, 16), (128, 128, 2, 16), (64, 64, 1, 32), (128, 128, 3, 32),
         (64, 128, 4, 32), (128, 64, 2, 32), (64, 64, 2, 64), (128, 64, 1, 64)]
# operand staging: 0 = registers + ds_write, 1/2 = LDS-DMA ring of depth 3/5 (bk 32 only)
# 3/4 = register staging with 2/4 K-groups of waves per block
# +8 = the same staging with the fp32-accurate split-bf16 (X6) math, +16 = X6 split once at the LDS
# store (bf16 planes, transposed LDS reads for K-major operands): held to the same f64 tolerance
VARIANTS = [0, 1, 2, 3, 4, 8, 9, 10, 11, 12, 16, 19, 20]
# +32 = bf16 operands, f32 accumulation (the engine's opt-in bf16 mode): bf16-level tolerance
VARIANTS += [32, 35, 36]
# +64 = F3: two fp16 planes of the power-of-two-scaled operand, 3 f16 MFMAs: held to the f64 tolerance
VARIANTS += [64, 67, 68]


def _tol(stage, f32=2e-5):
    return 2e-2 if stage & 32 else f32


def _stage_ok(stage, bm, bn, bk, conv0_fwd=False):
    """Python mirror of cs_conv_stage_ok (conv_gemm.hip) — used at collection time so the test
    matrix holds only combinations that have a kernel (a skip then always means a gap);
    test_stage_table_mirrors_kernel checks the mirror against the C++ function."""
    if sum(bool(stage & m) for m in (8, 16, 32, 64)) > 1:
        return False
    if stage & 64:
        stage &= ~64
        if conv0_fwd or stage not in (0, 3, 4):
            return False
        if bk == 64 and bm == 128 and bn == 128:
            return False
    if stage & 32:
        stage &= ~32
        if conv0_fwd or stage not in (0, 3, 4):
            return False
    if stage & 8:
        if conv0_fwd:
            return False
        stage &= ~8
    if stage & 16:
        stage &= ~16
        if conv0_fwd or stage not in (0, 3, 4):
            return False
        if bk == 64 and not (bm == 64 and bn == 64):
            return False
    if conv0_fwd and (stage != 0 or bk == 64):
        return False
    if stage == 0:
        return bk != 64 or not (bm == 128 and bn == 128)
    if stage == 1:
        return bk == 32
    if stage == 2:
        return bk == 32 and (bm + bn) * bk * 4 * 5 < 160 * 1024
    if stage == 3:
        return bk >= 32 and not (bk == 64 and bm == 128 and bn == 128)
    if stage == 4:
        return bk == 64 and not (bm == 128 and bn == 128)
    return False


def _matrix(shapes, tiles, conv0_fwd_shapes=()):
    return [pytest.param(sh, t, st, id=f"{sh}-{t}-{st}") for sh in shapes for t in tiles
            for st in VARIANTS if _stage_ok(st, t[0], t[1], t[3], sh in conv0_fwd_shapes)]


def _skip_stage(stage, bk, bm, bn, conv0_fwd=False):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    if not native.C().conv_stage_ok(stage, bm, bn, bk, conv0_fwd):
        pytest.fail(f"collected a combination with no kernel: stage {stage} / {bm}x{bn} / bk {bk}")


def test_stage_table_mirrors_kernel(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    for st in range(128):
        for bm in (64, 128):
            for bn in (64, 128):
                for bk in (16, 32, 64):
                    for c0 in (False, True):
                        assert _stage_ok(st, bm, bn, bk, c0) == C.conv_stage_ok(st, bm, bn, bk, c0), (st, bm, bn, bk, c0)


def _inputs(dev, B, H, cin, cout, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g, dtype=torch.float64)
    return x, w, b


def _nhwc(x, pad4=False):
    t = x.permute(0, 2, 3, 1)
    if pad4:
        t = F.pad(t, (0, 1))
    return t.contiguous()


@pytest.mark.parametrize("shape,tile,stage", _matrix(SHAPES, TILES, conv0_fwd_shapes=(SHAPES[0],)))
def test_conv_fwd_and_stats(dev, shape, tile, stage):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, sp, bk = tile
    _skip_stage(stage, bk, bm, bn, cin == 3)
    x, w, b = _inputs(dev, B, H, cin, cout)
    ref = F.conv2d(x, w, b, padding=1).permute(0, 2, 3, 1).reshape(-1, cout)
    conv0 = cin == 3
    xd = _nhwc(x, pad4=conv0).float().to(dev)
    wd = (w if conv0 else w.permute(0, 2, 3, 1)).contiguous().float().to(dev)
    y, st, rows = Fn.conv_fwd(xd, wd, b.float().to(dev), w_oihw=conv0, bm=bm, bn=bn, splits=sp, stats=True, bk=bk,
                            stage=stage)
    _close(y, ref, _tol(stage))
    M = ref.shape[0]
    for t in range(st.shape[0]):
        seg = ref[t * rows:min(M, (t + 1) * rows)]
        mu = seg.mean(0)
        _close(st[t, :, 0], mu, _tol(stage, 1e-4))
        _close(st[t, :, 1], ((seg - mu) ** 2).sum(0), _tol(stage, 1e-4))


@pytest.mark.parametrize("shape,tile,stage", _matrix(SHAPES[1:], TILES))
def test_conv_dgrad(dev, shape, tile, stage):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, sp, bk = tile
    _skip_stage(stage, bk, bm, bn)
    x, w, _ = _inputs(dev, B, H, cin, cout, 1)
    gy = torch.randn(B, cout, H, H, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_input(x.shape, w, gy, padding=1).permute(0, 2, 3, 1).reshape(-1, cin)
    dx = Fn.conv_dgrad(_nhwc(gy).float().to(dev).view(-1, cout), w.permute(0, 2, 3, 1).contiguous().float().to(dev),
                       B, H, H, bm=bm, bn=bn, splits=sp, bk=bk, stage=stage)
    _close(dx, ref, _tol(stage))


WGRAD_TILES = [(64, 64, 1, 16), (64, 64, 8, 16), (128, 128, 4, 16), (128, 64, 2, 16), (64, 64, 64, 16),
               (64, 128, 4, 32), (128, 128, 1, 32), (64, 64, 4, 64)]


@pytest.mark.parametrize("shape,tile,stage", _matrix(SHAPES, WGRAD_TILES))
def test_conv_wgrad(dev, shape, tile, stage):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, sp, bk = tile
    _skip_stage(stage, bk, bm, bn)
    x, w, _ = _inputs(dev, B, H, cin, cout, 2)
    gy = torch.randn(B, cout, H, H, dtype=torch.float64)
    ref = torch.nn.grad.conv2d_weight(x, w.shape, gy, padding=1)
    conv0 = cin == 3
    dw = Fn.conv_wgrad(_nhwc(gy).float().to(dev).view(-1, cout), _nhwc(x, pad4=conv0).float().to(dev), cout,
                       w_oihw=conv0, bm=bm, bn=bn, splits=sp, bk=bk, stage=stage)
    _close(dw, ref if conv0 else ref.permute(0, 2, 3, 1), _tol(stage))


@pytest.mark.parametrize("B,H,C,pool", [(2, 32, 64, True), (4, 8, 256, False), (3, 4, 512, True),
                                        (64, 2, 512, True), (5, 16, 128, True), (8, 8, 256, False),
                                        (16, 8, 256, False), (8, 4, 512, False), (64, 8, 256, False),
                                        (64, 32, 64, True)])
@pytest.mark.parametrize("fused", [False, True])
def test_bn_relu_pool_fwd_bwd(dev, B, H, C, pool, fused):
    # False: finalize / apply / reduce / finalize / apply launches; True: the single-launch kernels
    # (forward row-chunked over blocks)
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    torch.manual_seed(B * C)
    y = (torch.randn(B, C, H, H, dtype=torch.float64) * 2 + 0.5).requires_grad_()
    gamma = (torch.rand(C, dtype=torch.float64) + 0.5).requires_grad_()
    beta = torch.randn(C, dtype=torch.float64).requires_grad_()
    rm, rv = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    z = F.relu(F.batch_norm(y, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5))
    if pool:
        z = F.max_pool2d(z, 2, 2)
    G = torch.randn_like(z)
    z.backward(G)
    # device side: the conv epilogue's partials are emulated with one tile covering every row
    yd = _nhwc(y.detach()).float().to(dev).view(-1, C)
    mu = yd.double().mean(0)
    st = torch.stack([mu, ((yd.double() - mu) ** 2).sum(0)], 1).float()[None].contiguous()
    rmd, rvd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    gd, bd = gamma.detach().float().to(dev), beta.detach().float().to(dev)
    if fused:  # several partial tiles, to exercise the in-block Chan combine
        R = 16 if yd.shape[0] % 16 == 0 else yd.shape[0]
        seg = yd.double().view(-1, R, C)
        mu_t = seg.mean(1)
        st = torch.stack([mu_t, ((seg - mu_t[:, None]) ** 2).sum(1)], 2).float().contiguous()
        out, bst = Fn.bn_relu_pool_fwd(yd, st, R, B, H, H, gd, bd, rmd, rvd, nbt, pool=pool, fused=True)
        # every row chunk of the forward computed the same coefficients: bnv matches a fresh finalize
        _close(bst.mean, yd.double().mean(0), 1e-5)
    else:
        out, bst = Fn.bn_relu_pool_fwd(yd, st, yd.shape[0], B, H, H, gd, bd, rmd, rvd, nbt, pool=pool)
    _close(out, z.detach().permute(0, 2, 3, 1), 1e-5)
    _close(rmd, rm, 1e-5)
    _close(rvd, rv, 1e-5)
    assert int(nbt) == 1
    dz, dgamma, dbeta, dbias = Fn.bn_relu_pool_bwd(yd, _nhwc(G).float().to(dev), bst, gd, B, H, H, pool=pool,
                                                   fused=fused)
    _close(dz, y.grad.permute(0, 2, 3, 1).reshape(-1, C), 1e-4)
    _close(dgamma, gamma.grad, 1e-4)
    _close(dbeta, beta.grad, 1e-4)
    assert dbias.abs().max().item() <= 1e-3 * (beta.grad.abs().max().item() + 1)


def test_bn_eval(dev):
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, C = 3, 4, 128
    y = torch.randn(B, C, H, H, dtype=torch.float64)
    gamma, beta = torch.rand(C, dtype=torch.float64) + 0.5, torch.randn(C, dtype=torch.float64)
    rm, rv = torch.randn(C, dtype=torch.float64), torch.rand(C, dtype=torch.float64) + 0.2
    ref = F.max_pool2d(F.relu(F.batch_norm(y, rm, rv, gamma, beta, training=False, eps=1e-5)), 2, 2)
    f = lambda t: t.float().to(dev)  # noqa: E731
    out = Fn.bn_relu_pool_eval(_nhwc(y).float().to(dev).view(-1, C), B, H, H, f(gamma), f(beta), f(rm), f(rv),
                               pool=True)
    _close(out, ref.permute(0, 2, 3, 1), 1e-5)


@pytest.mark.parametrize("B,H,C,R", [(64, 32, 64, 16), (64, 32, 64, 7), (3, 32, 64, 1), (8, 16, 128, 2),
                                     (16, 16, 68, 2), (64, 16, 128, 16)])
def test_bn_finalize_many_partials(dev, B, H, C, R):
    # thousands of row-tile partials (conv0's 4096 at B=64): the 8-channel / 1024-thread finalize
    # (T >= 2048, C % 8 == 0), ragged last tiles, and the one-wave-per-channel fallback (C = 68)
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    torch.manual_seed(B * C + R)
    y = torch.randn(B, C, H, H, dtype=torch.float64) * 3 + 1.5
    gamma, beta = torch.rand(C, dtype=torch.float64) + 0.5, torch.randn(C, dtype=torch.float64)
    rm, rv = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    z = F.relu(F.batch_norm(y, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5))
    yd = _nhwc(y).float().to(dev).view(-1, C)
    M = yd.shape[0]
    T = (M + R - 1) // R
    yp = torch.cat([yd.double(), torch.zeros(T * R - M, C, dtype=torch.float64, device=dev)])
    cnt = torch.full((T,), float(R), dtype=torch.float64, device=dev)
    cnt[-1] = M - (T - 1) * R
    seg = yp.view(T, R, C)
    mu_t = seg.sum(1) / cnt[:, None]
    valid = (torch.arange(T * R, device=dev) < M).view(T, R, 1)
    m2_t = (((seg - mu_t[:, None]) ** 2) * valid).sum(1)
    st = torch.stack([mu_t, m2_t], 2).float().contiguous()
    rmd, rvd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    out, bst = Fn.bn_relu_pool_fwd(yd, st, R, B, H, H, gamma.float().to(dev), beta.float().to(dev), rmd, rvd, nbt,
                                   pool=False)
    _close(out, z.permute(0, 2, 3, 1), 1e-5)
    _close(bst.mean, y.mean((0, 2, 3)), 1e-5)
    _close(rmd, rm, 1e-5)
    _close(rvd, rv, 1e-5)
    assert int(nbt) == 1


# (B, H, cin, cout, tile): conv0 (1024 / 4096 row tiles: two-level combine), a 64x128 tile
# (128-channel column tiles), split-K (statistics from the combine's 16-row tiles), X6S K-groups
FIN_CASES = [((16, 32, 3, 64), (64, 64, 1, 16, 0)), ((64, 32, 3, 64), (64, 64, 1, 32, 0)),
             ((8, 16, 64, 128), (64, 128, 1, 32, 0)), ((8, 16, 64, 128), (128, 64, 1, 32, 3)),
             ((16, 8, 128, 256), (64, 64, 1, 64, 16 | 4)), ((16, 4, 256, 512), (64, 64, 3, 32, 0)),
             ((64, 2, 512, 512), (64, 64, 4, 64, 16 | 4)), ((5, 8, 128, 256), (64, 64, 2, 16, 0))]


@pytest.mark.parametrize("shape,tile", FIN_CASES)
def test_conv_fwd_in_launch_bn_finalize(dev, shape, tile):
    """The BN finalize done by the conv launch's last-arriving block (bn_fin.h: sc1 partials, two-level
    ticket combine) vs fp64 batch statistics of the same conv output: scale / shift / mean /
    invstd and the running-stat update; repeated launches leave the tickets zeroed and give the
    same bits (the combine order does not depend on which block arrives last)."""
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    B, H, cin, cout = shape
    bm, bn, sp, bk, stage = tile
    conv0 = cin == 3
    x, w, b = _inputs(dev, B, H, cin, cout, 3)
    x = x * 2.0 + 0.75  # a mean offset: the Chan combine must not lose the variance
    ref = F.conv2d(x, w, b, padding=1).permute(0, 2, 3, 1).reshape(-1, cout)
    xd = _nhwc(x, pad4=conv0).float().to(dev)
    wd = (w if conv0 else w.permute(0, 2, 3, 1)).contiguous().float().to(dev)
    g = torch.Generator().manual_seed(7)
    gamma = (torch.rand(cout, generator=g, dtype=torch.float64) + 0.5)
    beta = torch.randn(cout, generator=g, dtype=torch.float64)
    outs = []
    for _ in range(3):
        rm, rv = torch.full((cout,), 0.25, device=dev), torch.full((cout,), 2.0, device=dev)
        fin = dict(gamma=gamma.float().to(dev), beta=beta.float().to(dev), running_mean=rm, running_var=rv)
        y, st, rows, bs = Fn.conv_fwd(xd, wd, b.float().to(dev), w_oihw=conv0, bm=bm, bn=bn, splits=sp, stats=True,
                                      bk=bk, stage=stage, fin=fin)
        torch.cuda.synchronize()
        outs.append(torch.cat([bs.scale, bs.shift, bs.mean, bs.invstd, rm, rv]).cpu())
    mu, var = ref.mean(0), ref.var(0, unbiased=False)
    inv = 1.0 / torch.sqrt(var + 1e-5)
    _close(bs.mean, mu, 1e-5)
    _close(bs.invstd, inv, 1e-5)
    _close(bs.scale, gamma * inv, 1e-5)
    _close(bs.shift, beta - mu * gamma * inv, 1e-5)
    _close(rm, 0.9 * 0.25 + 0.1 * mu, 1e-5)
    _close(rv, 0.9 * 2.0 + 0.1 * ref.var(0, unbiased=True), 1e-5)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("B", [1, 4, 64])
def test_conv0_direct_kernels_match_fp64(dev, B):
    """VGG block 0 (3 -> 64, 3x3, pad 1) as the direct conv0.hip kernels: y (+bias), the BatchNorm
    tile statistics (per-tile mean and M2; the tile height is read off the statistics shape) and the OIHW weight gradient against float64
    PyTorch on the same inputs (channel 3 of the padded NHWC input is ignored)."""
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 32, 32, 4, generator=g)
    x[..., 3] = 7.0  # must not leak into the result
    w = torch.randn(64, 3, 3, 3, generator=g) * 0.2
    b = torch.randn(64, generator=g)
    y, st = C.conv0_fwd(x.to(dev), w.to(dev), b.to(dev), True)
    xr = x[..., :3].permute(0, 3, 1, 2).double()
    yr = F.conv2d(xr, w.double(), b.double(), padding=1).permute(0, 2, 3, 1).reshape(-1, 64)
    rel = (y.double().cpu() - yr).abs().max() / yr.abs().max()
    assert rel < 2e-6, rel
    rows = yr.shape[0] // st.shape[0]
    assert rows * st.shape[0] == yr.shape[0] and st.shape[1:] == (64, 2)
    t = yr.view(-1, rows, 64)
    mean = t.mean(1)
    m2 = ((t - mean[:, None, :]) ** 2).sum(1)
    st = st.double().cpu()
    assert ((st[..., 0] - mean).abs().max() / yr.abs().max()) < 2e-6
    assert ((st[..., 1] - m2).abs().max() / m2.abs().max()) < 2e-5
    dz = torch.randn(B * 1024, 64, generator=g)
    dw = C.conv0_wgrad(x.to(dev), dz.to(dev)).double().cpu()
    dzr = dz.double().view(B, 32, 32, 64).permute(0, 3, 1, 2)
    dwr = torch.nn.grad.conv2d_weight(xr, (64, 3, 3, 3), dzr, padding=1)
    assert ((dw - dwr).abs().max() / dwr.abs().max()) < 2e-5
    # deterministic: the fixed-order sum gives the same bits run to run
    assert torch.equal(C.conv0_wgrad(x.to(dev), dz.to(dev)).cpu(), dw.float())


@pytest.mark.parametrize("B", [1, 64])
def test_conv0_wgrad_bn_fold_bitwise(dev, B):
    """Block 0's weight gradient with its BN (+ReLU, 2x2 max-pool) backward apply folded in
    (`conv0_wgrad_bn`: dZ computed in LDS, never written) equals the separate BN backward
    (`bn_bwd`: reduce + finalize + apply -> dZ) followed by `conv0_wgrad`, bit for bit."""
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    g = torch.Generator().manual_seed(100 + B)
    x = torch.randn(B, 32, 32, 4, generator=g).to(dev)
    y = torch.randn(B * 1024, 64, generator=g).to(dev)
    G = torch.randn(B * 256, 64, generator=g).to(dev)
    gamma = (torch.rand(64, generator=g) + 0.5).to(dev)
    mean = (0.1 * torch.randn(64, generator=g)).to(dev)
    invstd = (torch.rand(64, generator=g) + 0.5).to(dev)
    scale = gamma * invstd
    shift = (0.2 * torch.randn(64, generator=g)).to(dev) - mean * scale
    part = torch.empty(C.bn_bwd_blocks(B, 32, 32, 64, True) * 64 * 3, device=dev)
    coef = torch.empty(64 * 3, device=dev)
    dz = torch.empty(B * 1024, 64, device=dev)
    C.bn_bwd(y, G, B, 32, 32, 64, True, scale, shift, mean, invstd, gamma, part, coef, None, None, None, dz)
    ref = C.conv0_wgrad(x, dz)
    fold = C.conv0_wgrad_bn(x, y, G, scale, shift, mean, invstd, coef)
    assert torch.equal(fold, ref), (fold - ref).abs().max()
    assert float(ref.abs().max()) > 0
