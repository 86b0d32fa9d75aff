"""The F3 conv math's error bounds (conv_gemm.hip "F3"), checked on the CPU with torch's IEEE
fp16 conversions standing in for v_cvt_f16_f32: each fp32 operand is scaled by the power of two
that puts its tensor maximum into [2^14, 2^15), split into h = fp16(x*2^s) and l = fp16(x*2^s - h),
and a product is taken as hl + lh + hh. The GPU kernels are held to the same f64 tolerance as the
X6S / f32 paths in tests/test_conv_bn_gpu.py and tests/test_native_engine_gpu.py; this pins the
arithmetic argument itself, and the shipped tile tables' use of it."""
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scale_exp(amax: float) -> int:
    e = torch.tensor(amax, dtype=torch.float32).view(torch.int32).item() >> 23 & 0xFF
    return 0 if e in (0, 255) else max(-100, min(100, 14 - (e - 127)))


def _split(x: torch.Tensor):
    s = _scale_exp(float(x.abs().max()))
    xs = x * (2.0 ** s)
    h = xs.half()
    l = (xs - h.float()).half()
    return h, l, s


def test_split_reconstructs_to_2e22():
    g = torch.Generator().manual_seed(0)
    for mag in (1e-9, 3e-4, 1.0, 7e3):
        # a spread of exponents inside one tensor (gradients span decades)
        x = torch.randn(1 << 16, generator=g) * mag * torch.exp(torch.randn(1 << 16, generator=g) * 3)
        h, l, s = _split(x)
        assert torch.isfinite(h).all() and torch.isfinite(l).all()
        assert float(h.float().abs().max()) < 2.0 ** 15 + 1
        back = (h.double() + l.double()) * 2.0 ** -s
        err = (back - x.double()).abs()
        # 2^-22 relative (l's rounding <= 2^-12 of |l| <= 2^-11 |x|), plus the fp16 subnormal floor
        # 2^-25 in scaled units = 2^-40 of the tensor maximum
        bound = 2.0 ** -22 * x.double().abs() + 2.0 ** -25 * 2.0 ** -s
        assert bool((err <= bound).all()), float((err / bound).max())


def test_three_product_dot_within_fp32_class_error():
    g = torch.Generator().manual_seed(1)
    K = 4608  # VGG-11's deepest 3x3 reduction (9 x 512)
    a = torch.randn(64, K, generator=g) * 0.05
    b = torch.randn(K, 64, generator=g) * 2e-5  # gradient-sized operand
    ah, al, sa = _split(a)
    bh, bl, sb = _split(b)
    d = lambda x: x.double()  # noqa: E731  (exact products; the MFMA accumulates in f32)
    c = (d(ah) @ d(bl) + d(al) @ d(bh) + d(ah) @ d(bh)) * 2.0 ** -(sa + sb)
    ref = a.double() @ b.double()
    mag = a.double().abs() @ b.double().abs()
    # dropped ll term and the splits' rounding: <= 2^-21 |a||b| per product
    assert float(((c - ref).abs() / mag).max()) <= 2.0 ** -21
    # the GPU tests' tolerance (2e-5 of the max |ref|) has ~50x margin on this bound
    assert float((c - ref).abs().max() / ref.abs().max()) < 2e-5 / 50


def test_shipped_tables_use_f3_only_where_it_has_a_kernel():
    """runtime/tiles_gfx950.json v3 = the v2 tiles with F3 on every X6S GEMM of blocks >= 1
    (scripts/make_f3_tables.py); F3 exists for register / K-group staging, not for 128x128 bk-64
    tiles, never for block 0 (its input has no producer-written bound)."""
    with open(os.path.join(ROOT, "cs744_pytorch_distributed_tutorial_amd", "runtime", "tiles_gfx950.json")) as f:
        db = json.load(f)
    v3 = [k for k in db if k.endswith("/gfx950/v3")]
    assert "VGG11/B64/gfx950/v3" in v3
    for k in v3:
        v2 = {tuple(t[:2]): t for t in db[k[:-2] + "v2"]["tiles"]}
        for t in db[k]["tiles"]:
            l, m, bm, bn, sp, bk = t[:6]
            st = t[6] if len(t) > 6 else 0
            old = v2[(l, m)]
            assert t[:6] == old[:6], (k, t, old)
            ost = old[6] if len(old) > 6 else 0
            if st & 64:
                assert l >= 1 and (st & ~64) in (0, 3, 4) and not (bk == 64 and bm == 128 and bn == 128), (k, t)
                assert ost == (st & ~64) | 16, (k, t, old)
            else:
                assert st == ost, (k, t, old)
