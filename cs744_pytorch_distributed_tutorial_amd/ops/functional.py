"""Tensor-level wrappers of the gfx950 conv / BatchNorm kernels (NHWC fp32).

These are the building blocks the native engine (``runtime.engine``) schedules
and the unit tests compare against PyTorch fp32 references. Layouts:

* activations NHWC ``[B, H, W, C]`` (the conv0 input is padded to 4 channels,
  channel 3 = 0, so every pixel is one float4);
* conv weights OHWI ``[Cout, 3, 3, Cin]`` (``w_ohwi``) — conv0 keeps torch's OIHW
  ``[64, 3, 3, 3]`` because its padded Cin differs from the stored one.

Reference ops replaced: ``nn.Conv2d(3x3, s1, p1, bias)`` -> ``nn.BatchNorm2d`` ->
``nn.ReLU(inplace)`` [-> ``nn.MaxPool2d(2, 2)``] (`master/part1/model.py:16-25`).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import native

FWD, DGRAD, WGRAD = 0, 1, 2
BN_EPS = 1e-5
BN_MOMENTUM = 0.1
SPLITK_STAT_ROWS = 16  # csrc/kernels/launchers.h CS_SPLITK_STAT_ROWS


def oihw_to_ohwi(w: torch.Tensor) -> torch.Tensor:
    return w.permute(0, 2, 3, 1).contiguous()


def ohwi_to_oihw(w: torch.Tensor) -> torch.Tensor:
    return w.permute(0, 3, 1, 2).contiguous()


def gemm_dims(mode: int, B: int, H: int, W: int, cin: int, cout: int) -> Tuple[int, int, int]:
    pix = B * H * W
    if mode == FWD:
        return pix, cout, 9 * cin
    if mode == DGRAD:
        return pix, cin, 9 * cout
    return cout, 9 * cin, pix


def _ws(mode, B, H, W, cin, cout, splits, device) -> Optional[torch.Tensor]:
    if splits <= 1:
        return None
    M, N, K = gemm_dims(mode, B, H, W, cin, cout)
    return torch.empty(splits * M * N, device=device, dtype=torch.float32)


def _counters(fixup: bool, mode, B, H, W, cin, cout, bm, bn, device) -> Optional[torch.Tensor]:
    """Zeroed split-K tile tickets for the in-launch combine (``fixup``), one per output tile."""
    if not fixup:
        return None
    M, N, _ = gemm_dims(mode, B, H, W, cin, cout)
    return torch.zeros(((M + bm - 1) // bm) * ((N + bn - 1) // bn), device=device, dtype=torch.int32)


def conv_fwd(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], *, w_oihw: bool = False,
             bm: int = 64, bn: int = 64, splits: int = 1, stats: bool = False, bk: int = 16, fixup: bool = False,
             stage: int = 0):
    """y[B*H*W, Cout] = conv3x3(x NHWC) (+bias); optionally per-tile (mean, M2) BN partials.
    ``fixup``: split-K slabs combined in-launch by each tile's last block (no reduce kernel)."""
    B, H, W, cin = x.shape
    cout = w.shape[0]
    y = torch.empty(B * H * W, cout, device=x.device, dtype=torch.float32)
    R = native.C().conv_stat_rows(9 * cin, bm, bn, bk, splits, fixup)
    T = (B * H * W + R - 1) // R
    st = torch.empty(T, cout, 2, device=x.device, dtype=torch.float32) if stats else None
    rows = native.C().conv_gemm(FWD, x, w, None, bias, y, _ws(FWD, B, H, W, cin, cout, splits, x.device), st,
                                B, H, W, cin, cout, w_oihw, bm, bn, splits, bk,
                                _counters(fixup, FWD, B, H, W, cin, cout, bm, bn, x.device), stage)
    return (y, st, rows) if stats else y


def conv_dgrad(dz: torch.Tensor, w_ohwi: torch.Tensor, B: int, H: int, W: int, *, bm: int = 64, bn: int = 64,
               splits: int = 1, bk: int = 16, fixup: bool = False, stage: int = 0) -> torch.Tensor:
    """dx[B*H*W, Cin] from dz[B*H*W, Cout] and OHWI weights."""
    cout, _, _, cin = w_ohwi.shape
    dx = torch.empty(B * H * W, cin, device=dz.device, dtype=torch.float32)
    native.C().conv_gemm(DGRAD, None, w_ohwi, dz, None, dx, _ws(DGRAD, B, H, W, cin, cout, splits, dz.device), None,
                         B, H, W, cin, cout, False, bm, bn, splits, bk,
                         _counters(fixup, DGRAD, B, H, W, cin, cout, bm, bn, dz.device), stage)
    return dx


def conv_wgrad(dz: torch.Tensor, x: torch.Tensor, cout: int, *, w_oihw: bool = False, bm: int = 64, bn: int = 64,
               splits: int = 1, bk: int = 16, fixup: bool = False, stage: int = 0) -> torch.Tensor:
    """dW (OHWI, or OIHW [Cout,3,3,3] for the padded conv0) from dz and the NHWC input."""
    B, H, W, cin = x.shape
    dw = torch.empty(cout * 27 if w_oihw else cout * 9 * cin, device=x.device, dtype=torch.float32)
    native.C().conv_gemm(WGRAD, x, None, dz, None, dw, _ws(WGRAD, B, H, W, cin, cout, splits, x.device), None,
                         B, H, W, cin, cout, w_oihw, bm, bn, splits, bk,
                         _counters(fixup, WGRAD, B, H, W, cin, cout, bm, bn, x.device), stage)
    return dw.view(cout, 3, 3, 3) if w_oihw else dw.view(cout, 3, 3, cin)


def split3(t: torch.Tensor) -> torch.Tensor:
    """fp32 tensor -> P3 bf16 chunks ``[numel/8, 3, 8]`` (h, m, l of every 8 elements, t = h + m + l
    to 2^-26 |t|): the operand format of the pre-split ("XP") conv GEMMs
    (``csrc/kernels/conv_xp.hip``)."""
    t = t.contiguous()
    out = torch.empty(t.numel() // 8, 3, 8, device=t.device, dtype=torch.bfloat16)
    native.C().split3(t, out)
    return out


def conv_fwd_xp(x3: torch.Tensor, w3: torch.Tensor, bias: Optional[torch.Tensor], B: int, H: int, W: int, cin: int,
                cout: int, *, bm: int = 128, bn: int = 64, bk: int = 32, kg: int = 1, splits: int = 1,
                stats: bool = False, nb: int = 0):
    """``conv_fwd`` on pre-split operands: x3 = split3(x NHWC), w3 = split3(w OHWI)."""
    y = torch.empty(B * H * W, cout, device=x3.device, dtype=torch.float32)
    R = native.C().conv_stat_rows(9 * cin, bm, bn, bk, splits, False)
    T = (B * H * W + R - 1) // R
    st = torch.empty(T, cout, 2, device=x3.device, dtype=torch.float32) if stats else None
    rows = native.C().conv_gemm_xp(FWD, x3, w3, None, bias, y, _ws(FWD, B, H, W, cin, cout, splits, x3.device), st,
                                   B, H, W, cin, cout, bm, bn, splits, bk, kg, nb)
    return (y, st, rows) if stats else y


def conv_dgrad_xp(dz3: torch.Tensor, w3: torch.Tensor, B: int, H: int, W: int, cin: int, cout: int, *,
                  bm: int = 128, bn: int = 64, bk: int = 32, kg: int = 1, splits: int = 1,
                  nb: int = 0) -> torch.Tensor:
    dx = torch.empty(B * H * W, cin, device=dz3.device, dtype=torch.float32)
    native.C().conv_gemm_xp(DGRAD, None, w3, dz3, None, dx, _ws(DGRAD, B, H, W, cin, cout, splits, dz3.device), None,
                            B, H, W, cin, cout, bm, bn, splits, bk, kg, nb)
    return dx


def conv_wgrad_xp(dz3: torch.Tensor, x3: torch.Tensor, B: int, H: int, W: int, cin: int, cout: int, *,
                  bm: int = 128, bn: int = 64, bk: int = 32, kg: int = 1, splits: int = 1,
                  nb: int = 0) -> torch.Tensor:
    dw = torch.empty(cout * 9 * cin, device=x3.device, dtype=torch.float32)
    native.C().conv_gemm_xp(WGRAD, x3, None, dz3, None, dw, _ws(WGRAD, B, H, W, cin, cout, splits, x3.device), None,
                            B, H, W, cin, cout, bm, bn, splits, bk, kg, nb)
    return dw.view(cout, 3, 3, cin)


_GRID_BARS = {}


def _grid_bar(device) -> torch.Tensor:
    """Zeroed grid-barrier counters of the one-launch BN kernels (left zeroed by every launch)."""
    key = str(device)
    if key not in _GRID_BARS:
        _GRID_BARS[key] = torch.zeros(640, dtype=torch.int32, device=device)  # kCsBnGridBarInts
    return _GRID_BARS[key]


class BNState:
    """Per-channel tensors one BN layer needs between forward and backward."""

    def __init__(self, C: int, device):
        f = dict(device=device, dtype=torch.float32)
        self.scale = torch.empty(C, **f)
        self.shift = torch.empty(C, **f)
        self.mean = torch.empty(C, **f)
        self.invstd = torch.empty(C, **f)


def bn_relu_pool_fwd(y: torch.Tensor, stats: torch.Tensor, rows: int, B: int, H: int, W: int, gamma, beta,
                     running_mean=None, running_var=None, nbt=None, pool: bool = False,
                     momentum: float = BN_MOMENTUM, eps: float = BN_EPS, fused: bool = False):
    """Training-mode BN (batch stats from the conv epilogue partials) + ReLU (+2x2 max-pool).
    ``fused``: the single-launch kernel (one block per 16 channels; the engine's small layers)."""
    C = gamma.numel()
    M = B * H * W
    T = stats.shape[0]
    if fused == "grid":  # one grid-barrier launch (the engine's default for the larger layers)
        bnv = torch.empty(4, C, device=y.device, dtype=torch.float32)
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        out = torch.empty(B, Ho, Wo, C, device=y.device, dtype=torch.float32)
        native.C().bn_grid_fwd(stats, T, rows, M, gamma, beta, running_mean, running_var, nbt, momentum, eps, bnv,
                               y, out, B, H, W, pool, _grid_bar(y.device))
        st = BNState(C, y.device)
        st.scale, st.shift, st.mean, st.invstd = bnv[0], bnv[1], bnv[2], bnv[3]
        return out, st
    if fused:
        bnv = torch.empty(4, C, device=y.device, dtype=torch.float32)
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        out = torch.empty(B, Ho, Wo, C, device=y.device, dtype=torch.float32)
        native.C().bn_fused_fwd(stats, T, rows, M, gamma, beta, running_mean, running_var, nbt, momentum, eps, bnv,
                                y, out, B, H, W, pool)
        st = BNState(C, y.device)
        st.scale, st.shift, st.mean, st.invstd = bnv[0], bnv[1], bnv[2], bnv[3]
        return out, st
    st = BNState(C, y.device)
    native.C().bn_finalize(stats, T, rows, M, gamma, beta, running_mean, running_var, nbt, momentum, eps,
                           st.scale, st.shift, st.mean, st.invstd)
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    out = torch.empty(B, Ho, Wo, C, device=y.device, dtype=torch.float32)
    native.C().bn_apply(y, st.scale, st.shift, out, B, H, W, C, pool)
    return out, st


def bn_relu_pool_eval(y: torch.Tensor, B: int, H: int, W: int, gamma, beta, running_mean, running_var,
                      pool: bool = False, eps: float = BN_EPS) -> torch.Tensor:
    C = gamma.numel()
    scale = torch.empty(C, device=y.device)
    shift = torch.empty(C, device=y.device)
    native.C().bn_eval_coeffs(gamma, beta, running_mean, running_var, eps, scale, shift)
    Ho, Wo = (H // 2, W // 2) if pool else (H, W)
    out = torch.empty(B, Ho, Wo, C, device=y.device, dtype=torch.float32)
    native.C().bn_apply(y, scale, shift, out, B, H, W, C, pool)
    return out


def bn_relu_pool_bwd(y: torch.Tensor, G: torch.Tensor, st: BNState, gamma: torch.Tensor, B: int, H: int, W: int,
                     pool: bool = False, fused: bool = False):
    """-> (dz [B*H*W, C], dgamma, dbeta, dbias) for z = maxpool?(relu(bn(y))).
    ``fused``: True = one launch (small layers), "two" = chunk partials + finalize-in-apply."""
    C = gamma.numel()
    if fused == "grid":
        bnv = torch.stack([st.scale, st.shift, st.mean, st.invstd]).contiguous()
        part = torch.empty(native.C().bn_bwd_blocks(B, H, W, C, pool) * C * 3, device=y.device)
        coef = torch.empty(C * 3, device=y.device)
        dgamma, dbeta, dbias = (torch.empty(C, device=y.device) for _ in range(3))
        dz = torch.empty(B * H * W, C, device=y.device)
        native.C().bn_grid_bwd(y, G, B, H, W, C, pool, bnv, gamma, part, coef, dgamma, dbeta, dbias, dz,
                               _grid_bar(y.device))
        return dz, dgamma, dbeta, dbias
    if fused == "two":
        bnv = torch.stack([st.scale, st.shift, st.mean, st.invstd]).contiguous()
        part = torch.empty(native.C().bn_bwd_chunks(B, H, W, C, pool) * C * 3, device=y.device)
        dgamma, dbeta, dbias = (torch.empty(C, device=y.device) for _ in range(3))
        dz = torch.empty(B * H * W, C, device=y.device)
        native.C().bn_bwd2(y, G, B, H, W, C, pool, bnv, gamma, part, dgamma, dbeta, dbias, dz)
        return dz, dgamma, dbeta, dbias
    if fused:
        bnv = torch.stack([st.scale, st.shift, st.mean, st.invstd]).contiguous()
        coef = torch.empty(C * 3, device=y.device)
        dgamma, dbeta, dbias = (torch.empty(C, device=y.device) for _ in range(3))
        dz = torch.empty(B * H * W, C, device=y.device)
        native.C().bn_fused_bwd(y, G, B, H, W, C, pool, bnv, gamma, coef, dgamma, dbeta, dbias, dz)
        return dz, dgamma, dbeta, dbias
    P = native.C().bn_bwd_blocks(B, H, W, C, pool)
    part = torch.empty(P * C * 3, device=y.device)
    coef = torch.empty(C * 3, device=y.device)
    dgamma = torch.empty(C, device=y.device)
    dbeta = torch.empty(C, device=y.device)
    dbias = torch.empty(C, device=y.device)
    dz = torch.empty(B * H * W, C, device=y.device)
    native.C().bn_bwd(y, G, B, H, W, C, pool, st.scale, st.shift, st.mean, st.invstd, gamma, part, coef, dgamma,
                      dbeta, dbias, dz)
    return dz, dgamma, dbeta, dbias
