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


def conv_fwd(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], *, w_oihw: bool = False,
             bm: int = 64, bn: int = 64, splits: int = 1, stats: bool = False, bk: int = 16, stage: int = 0,
             fin: Optional[dict] = None):
    """y[B*H*W, Cout] = conv3x3(x NHWC) (+bias); optionally per-tile (mean, M2) BN partials.
    ``fin`` (needs ``stats``): the BN finalize by the launch's last-arriving block (bn_fin.h), a
    dict of gamma, beta and optional running_mean / running_var / momentum / eps; the result
    then carries ``BNState`` as a 4th element (scale, shift, mean, invstd)."""
    B, H, W, cin = x.shape
    cout = w.shape[0]
    y = torch.empty(B * H * W, cout, device=x.device, dtype=torch.float32)
    R = native.C().conv_stat_rows(9 * cin, bm, bk, splits)
    T = (B * H * W + R - 1) // R
    st = torch.empty(T, cout, 2, device=x.device, dtype=torch.float32) if stats else None
    kw = {}
    bnv = None
    if fin is not None:
        M, _, K = gemm_dims(FWD, B, H, W, cin, cout)
        nsp = native.C().conv_effective_splits(K, bk, splits)
        ints, grp = native.C().bn_fin_sizes(T, cout, 64 if nsp > 1 else bn)
        bnv = torch.empty(4, cout, device=x.device, dtype=torch.float32)
        kw = dict(fin_cnt=torch.zeros(ints, device=x.device, dtype=torch.int32),
                  fin_grp=torch.empty(max(grp, 4), device=x.device, dtype=torch.float32),
                  gamma=fin["gamma"], beta=fin["beta"], running_mean=fin.get("running_mean"),
                  running_var=fin.get("running_var"), bnv=bnv, momentum=fin.get("momentum", BN_MOMENTUM),
                  eps=fin.get("eps", BN_EPS))
    kw.update(_f3_amax(stage, x, w))
    rows = native.C().conv_gemm(FWD, x, w, None, bias, y, _ws(FWD, B, H, W, cin, cout, splits, x.device), st,
                                B, H, W, cin, cout, w_oihw, bm, bn, splits, bk, stage, **kw)
    if bnv is not None:
        bs = BNState(cout, x.device)
        bs.scale, bs.shift, bs.mean, bs.invstd = bnv[0], bnv[1], bnv[2], bnv[3]
        return y, st, rows, bs
    return (y, st, rows) if stats else y


def conv_dgrad(dz: torch.Tensor, w_ohwi: torch.Tensor, B: int, H: int, W: int, *, bm: int = 64, bn: int = 64,
               splits: int = 1, bk: int = 16, stage: int = 0) -> torch.Tensor:
    """dx[B*H*W, Cin] from dz[B*H*W, Cout] and OHWI weights."""
    cout, _, _, cin = w_ohwi.shape
    dx = torch.empty(B * H * W, cin, device=dz.device, dtype=torch.float32)
    native.C().conv_gemm(DGRAD, None, w_ohwi, dz, None, dx, _ws(DGRAD, B, H, W, cin, cout, splits, dz.device), None,
                         B, H, W, cin, cout, False, bm, bn, splits, bk, stage, **_f3_amax(stage, dz, w_ohwi))
    return dx


def conv_wgrad(dz: torch.Tensor, x: torch.Tensor, cout: int, *, w_oihw: bool = False, bm: int = 64, bn: int = 64,
               splits: int = 1, bk: int = 16, stage: int = 0) -> torch.Tensor:
    """dW (OHWI, or OIHW [Cout,3,3,3] for the padded conv0) from dz and the NHWC input."""
    B, H, W, cin = x.shape
    dw = torch.empty(cout * 27 if w_oihw else cout * 9 * cin, device=x.device, dtype=torch.float32)
    native.C().conv_gemm(WGRAD, x, None, dz, None, dw, _ws(WGRAD, B, H, W, cin, cout, splits, x.device), None,
                         B, H, W, cin, cout, w_oihw, bm, bn, splits, bk, stage, **_f3_amax(stage, dz, x))
    return dw.view(cout, 3, 3, 3) if w_oihw else dw.view(cout, 3, 3, cin)


STAGE_F3 = 64  # launchers.h CS_STAGE_F3
AMAX_SLOT = 64 * 32  # launchers.h CS_AMAX_SLOT


def _f3_amax(stage: int, a: torch.Tensor, b: torch.Tensor) -> dict:
    """The F3 stage's operand bounds (conv_gemm.hip "F3"): |A|max and |B|max as one-float tensors
    (the engine has them from the operands' producers; here torch computes them)."""
    if not stage & STAGE_F3:
        return {}
    # one slot of CS_AMAX_SLOT (64 shards x 32) floats each: the kernel takes the largest shard
    return dict(amax_a=a.detach().abs().max().reshape(1).float().repeat(AMAX_SLOT),
                amax_b=b.detach().abs().max().reshape(1).float().repeat(AMAX_SLOT))


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
    ``fused``: one launch (reduce + finalize + apply; the engine's small top layer)."""
    C = gamma.numel()
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
