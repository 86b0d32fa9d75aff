"""Channels-last (NHWC) convolution, BatchNorm(+residual)(+ReLU) and 3x3/2 max-pool for the
ResNet family's native path (``csrc/kernels/cnn_nhwc.hip``; models/resnet.py ``layout="nhwc"``).

Activations are contiguous ``[B, H, W, C]`` tensors (fp32, or bf16 under autocast). A bf16
convolution with C, Cout % 32 == 0 that is not a plain 1x1/stride-1 one runs as the gfx950
implicit-GEMM kernel (``csrc/kernels/conv_nhwc.hip``: forward, data and weight gradient gather
their operands straight from the activations, no patch matrix in memory), and so does the
4-channel stem (its C4 mode); the others are one
GEMM on MI355X's matrix cores (hipBLASLt via ``torch.mm``):

* 1x1 / stride 1: the activation *is* the ``[B*H*W, Cin]`` operand, no copy;
* anything else (3x3, the 7x7 stem, strided 1x1 shortcuts): the gfx950 ``im2col_nhwc`` gather
  builds ``[B*Ho*Wo, Kp]`` (columns ordered (r, s, c), K padded to a 16-byte multiple), kept
  for the weight gradient; the data gradient is ``dcol = dy @ W`` folded back by the
  gather-style ``col2im_nhwc`` (deterministic, no atomics).

No NCHW<->NHWC transposes anywhere in the step (MIOpen's NCHW path spends ~20 % of a ResNet-50
bf16 step in them, ``profiles/r2_resnet50_bf16_kernels.txt``). BatchNorm follows
``nn.BatchNorm2d`` training semantics (batch statistics, biased variance for normalisation,
unbiased for the running variance, ``num_batches_tracked`` += 1); eval mode and CPU tensors use
the module's running statistics through plain torch ops.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import native


def act_dtype(x: torch.Tensor) -> torch.dtype:
    """bf16 under CUDA autocast (its dtype), else the input's dtype"""
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


def to_nhwc(x: torch.Tensor, dtype: Optional[torch.dtype] = None, pad_c: int = 0) -> torch.Tensor:
    """[B, C, H, W] (any memory format) -> contiguous [B, H, W, C (+ pad_c zero channels)]"""
    x = x.permute(0, 2, 3, 1)
    if dtype is not None:
        x = x.to(dtype)
    return F.pad(x, (0, pad_c)).contiguous() if pad_c else x.contiguous()


def _kpad(k: int, dtype: torch.dtype) -> int:
    v = 8 if dtype == torch.bfloat16 else 4
    return (k + v - 1) // v * v


def _wgrad_splits(M: int, Co: int, Kp: int) -> int:
    """row chunks for the weight-gradient GEMM dW = dY^T @ col ([Co, M] x [M, Kp]): its output is
    small and its reduction long (M = B*Ho*Wo rows: 401k for ResNet-50's first stage at B=128), so
    one GEMM fills few of the 256 CUs (hipBLASLt measured ~30 TFLOP/s on it); S chunks run as one
    batched GEMM with fp32 partials, summed after"""
    tiles = max(1, (Co // 128) * (Kp // 128))
    s = 1
    while s < 64 and tiles * s * 2 <= 1024 and M % (2 * s) == 0 and M // (2 * s) >= 2048:
        s *= 2
    return s


# GEMMs of the im2col / 1x1 convolutions: "blas" = torch.mm (hipBLASLt), "native" = the gfx950
# bf16 GEMM of csrc/kernels/gemm_bf16.hip for every bf16 one (operands read in place, transposed in
# LDS where needed, split-K weight gradient), "auto" = native where the output has >= 256 columns
# (its 256 x 256 tile would be mostly idle on narrower ones), "wgrad" = native for the weight
# gradients with >= 256 rows and columns only (dY^T col, both operands M-major: the product where
# the native GEMM beats hipBLASLt, profiles/r4_gemm_bench_v2.jsonl; ops/lm.py's CS_LM_GEMM=wgrad)
_CONV_GEMM = os.environ.get("CS_CONV_GEMM", "blas")
if _CONV_GEMM not in ("blas", "native", "auto", "wgrad"):
    raise ValueError(f"CS_CONV_GEMM must be 'blas', 'native', 'auto' or 'wgrad', got {_CONV_GEMM!r}")


def _native_gemm(a: torch.Tensor, n: int, wgrad: bool = False, m: int = 0) -> bool:
    if a.dtype != torch.bfloat16:
        return False
    return (_CONV_GEMM == "native" or (_CONV_GEMM == "auto" and n >= 256)
            or (_CONV_GEMM == "wgrad" and wgrad and n >= 256 and m >= 256))


# a native-GEMM forward convolution also returns its output's BatchNorm statistics per 256-row
# tile (the GEMM epilogue, gemm_bf16.hip tile_stats); the BatchNorm reading that output then skips
# its statistics pass (cs_bn_nhwc_fwd_tiles)
_BN_STATS = True


def _wgrad(dy2: torch.Tensor, col: torch.Tensor) -> torch.Tensor:
    """fp32 dY^T @ col, split over row chunks when the output alone cannot fill the chip"""
    M, Co = dy2.shape
    Kp = col.shape[1]
    if _native_gemm(col, Kp, wgrad=True, m=Co):
        return native.C().mm_bf16(dy2.t(), col, True)  # split-K slabs + fixed-order sum inside
    S = _wgrad_splits(M, Co, Kp)
    if S == 1:
        return torch.mm(dy2.t(), col, out_dtype=torch.float32) if col.dtype != torch.float32 else torch.mm(dy2.t(), col)
    a = dy2.view(S, M // S, Co).transpose(1, 2)
    b = col.view(S, M // S, Kp)
    part = torch.bmm(a, b, out_dtype=torch.float32) if col.dtype != torch.float32 else torch.bmm(a, b)
    if Co * Kp % 4 == 0:
        return native.C().slab_sum(part)  # split-lane slab sum (csrc/kernels/conv_nhwc.hip)
    return part.sum(0)


def _weight_grad(v: torch.Tensor, ctx) -> torch.Tensor:
    """a [Co, Ci, R, S] view of a GEMM's fp32 weight gradient -> the gradient in the weight's own
    layout (autograd would otherwise copy it to match): the view itself when it already is that
    layout, else one copy into it"""
    if v.dtype == ctx.wdtype and v.stride() == ctx.wstride:
        return v
    dw = torch.empty_strided(v.shape, ctx.wstride, dtype=ctx.wdtype, device=v.device)
    dw.copy_(v)
    return dw


def _implicit_ok(dt: torch.dtype, C: int, Ci: int, Co: int, R: int, S: int, stride: int, pad: int) -> bool:
    """whether this conv runs as the bf16 implicit-GEMM kernel (csrc/kernels/conv_nhwc.hip).

    It serves every bf16 conv with C, Cout % 32 == 0 (not the 4-channel stem; plain 1x1/stride-1
    convs already are a GEMM on the activation). By default it takes the stride-1 convs with at
    most 128 input channels — the memory-bound ones, where not writing and re-reading the patch
    matrix wins: ResNet-50 at B=256, fwd+bwd per conv, 56x56x64 3x3 681 vs 1545 us and 28x28x128
    3x3 603 vs 855 us; the deeper, compute-bound convs stay on im2col + hipBLASLt, which is faster
    there (14x14x256 3x3 421 vs 615 us; profiles/r3_conv_nhwc_bench.jsonl).
    CS_CONV_IMPLICIT: 0 never, 1 (default) that policy, 2 every conv it serves."""
    mode = os.environ.get("CS_CONV_IMPLICIT", "1")
    if mode == "0" or dt != torch.bfloat16 or C != Ci or Ci % 32 or Co % 32:
        return False
    if R == 1 and S == 1 and stride == 1 and pad == 0:
        return False
    return mode == "2" or (stride == 1 and Ci <= 128)


class _ConvImplicitNHWC(torch.autograd.Function):
    """bf16 implicit-GEMM convolution (csrc/kernels/conv_nhwc.hip): no patch matrix in memory
    forward or backward; saves x and the [Co, R, S, C] weight"""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int):
        Co, Ci, R, S = weight.shape
        w4 = weight.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()  # [Co, R, S, C]
        y = native.C().conv_nhwc_bf16(0, x, w4, R, S, stride, pad, 0, 0)
        ctx.save_for_backward(x, w4)
        ctx.geo = (R, S, stride, pad)
        ctx.wdtype = weight.dtype
        ctx.wstride = weight.stride()
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w4 = ctx.saved_tensors
        R, S, stride, pad = ctx.geo
        dy = dy.to(torch.bfloat16).contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = w4.permute(3, 1, 2, 0).contiguous()  # [C, R, S, Co]
            dx = native.C().conv_nhwc_bf16(1, dy, wt, R, S, stride, pad, x.shape[1], x.shape[2])
        if ctx.needs_input_grad[1]:
            dwf = native.C().conv_nhwc_bf16(2, dy, x, R, S, stride, pad, 0, 0)  # fp32 [Co, R*S*C]
            Co, C = w4.shape[0], w4.shape[3]
            dw = _weight_grad(dwf.view(Co, R, S, C).permute(0, 3, 1, 2), ctx)
        return dx, dw, None, None


def _stem_ok(x: torch.Tensor, Ci: int, Co: int, S: int) -> bool:
    """the 4-channel stem (image + a zero channel) as the implicit-GEMM kernel's C4 mode: forward and
    weight gradient without the [B*Ho*Wo, R*S*4] patch matrix (1.3 GB for ResNet-50 at B=256, written
    by im2col and read twice). The image needs no gradient. CS_CONV_IMPLICIT=0 disables."""
    return (os.environ.get("CS_CONV_IMPLICIT", "1") != "0"
            and act_dtype(x) == torch.bfloat16 and x.shape[3] == 4
            and Ci <= 4 and S <= 8 and Co % 32 == 0 and not x.requires_grad)


class _ConvStemNHWC(torch.autograd.Function):
    """C4 mode of csrc/kernels/conv_nhwc.hip: kernel rows padded to 8 taps of 4 channels (K = R*32),
    weight [Co, R, 8, 4]; saves only the image"""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int):
        Co, Ci, R, S = weight.shape
        w4 = F.pad(weight.permute(0, 2, 3, 1), (0, 4 - Ci, 0, 8 - S)).to(torch.bfloat16).contiguous()
        y = native.C().conv_nhwc_bf16(0, x, w4, R, S, stride, pad, 0, 0)
        ctx.save_for_backward(x)
        ctx.geo = (Co, Ci, R, S, stride, pad)
        ctx.wdtype = weight.dtype
        ctx.wstride = weight.stride()
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        Co, Ci, R, S, stride, pad = ctx.geo
        dw = None
        if ctx.needs_input_grad[1]:
            dwf = native.C().conv_nhwc_bf16(2, dy.to(torch.bfloat16).contiguous(), x, R, S, stride, pad, 0, 0)
            dw = _weight_grad(dwf.view(Co, R, 8, 4)[:, :, :S, :Ci].permute(0, 3, 1, 2), ctx)
        return None, dw, None, None


class ResidualGradSink(torch.autograd.Function):
    """Identity on the residual branch of a block whose first conv is a plain 1x1 (ResNet
    bottleneck): the residual's gradient is handed to that conv's backward through ``box``, which
    adds it in its data-gradient GEMM (``addmm``, beta = 1) instead of autograd summing the two
    gradients of the block input in a separate elementwise pass (3 activation-sized passes -> 1).
    Whichever of the two backward nodes runs first decides: if the conv's backward already ran,
    this one returns the gradient itself and autograd adds as usual."""

    @staticmethod
    def forward(ctx, x, box: dict):
        ctx.box = box
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        if box.get("done"):
            return g, None
        box["g"] = g
        return None, None


class _ConvNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int, box: Optional[dict] = None):
        B, H, W, C = x.shape
        Co, Ci, R, S = weight.shape
        # x may carry zero channels beyond the weight's (the stem's 3 -> 4, for vector access)
        assert Ci <= C, f"conv_nhwc: {C} input channels for a {Ci}-channel weight"
        Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        K = R * S * C
        w4 = weight.permute(0, 2, 3, 1)
        if Ci < C:
            w4 = F.pad(w4, (0, C - Ci))
        wf = w4.reshape(Co, K).to(x.dtype)  # [Co, K], columns (r, s, c)
        direct = R == 1 and S == 1 and stride == 1 and pad == 0
        if direct:
            col = x.view(B * H * W, C)
        else:
            Kp = _kpad(K, x.dtype)
            col = native.C().im2col_nhwc(x, R, S, stride, pad, Kp)
            if Kp != K:
                wf = F.pad(wf, (0, Kp - K))
        wf = wf.contiguous()
        tiles = None
        with torch.autocast("cuda", enabled=False):
            if _native_gemm(col, Co) and _BN_STATS:
                y, tiles = native.C().mm_bf16_bn_stats(col, wf.t())
                ctx.mark_non_differentiable(tiles)
            elif _native_gemm(col, Co):
                y = native.C().mm_bf16(col, wf.t())
            else:
                y = torch.mm(col, wf.t())
        ctx.save_for_backward(col, wf)
        ctx.geo = (B, H, W, C, Ci, Co, R, S, stride, pad, K, direct)
        ctx.wdtype = weight.dtype
        ctx.wstride = weight.stride()
        ctx.box = box
        if tiles is not None:
            return y.view(B, Ho, Wo, Co), tiles
        return y.view(B, Ho, Wo, Co)

    @staticmethod
    def backward(ctx, dy, *_tiles):
        col, wf = ctx.saved_tensors
        B, H, W, C, Ci, Co, R, S, stride, pad, K, direct = ctx.geo
        dy2 = dy.reshape(-1, Co)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = None
        with torch.autocast("cuda", enabled=False):
            if ctx.needs_input_grad[1]:
                dwf = _wgrad(dy2, col)  # [Co, Kp] fp32
                # a fresh standard-strided [Co, Ci, R, S] tensor (a permuted view of a 1x1 kernel would
                # pass is_contiguous() with non-standard strides for its size-1 dims)
                if R == 1 and S == 1 and dwf.shape[1] == K and Ci == C:
                    dw = dwf.view(Co, C, 1, 1).to(ctx.wdtype)
                else:
                    dw = _weight_grad(dwf[:, :K].reshape(Co, R, S, C)[..., :Ci].permute(0, 3, 1, 2), ctx)
            if ctx.needs_input_grad[0]:
                assert Ci == C, "conv_nhwc: no data gradient through padded input channels"
                box = ctx.box
                gres = box.pop("g", None) if box is not None and direct else None
                if box is not None:
                    box["done"] = True  # a ResidualGradSink running after this returns its gradient
                    box["fused"] = gres is not None
                nat = _native_gemm(dy2, wf.shape[1])
                if gres is not None and gres.dtype == dy2.dtype and gres.is_contiguous():
                    # dx + the residual's gradient in one GEMM (beta = 1), written over the residual
                    # gradient itself (an out-of-place addmm would first copy it into a new buffer)
                    dcol = native.C().mm_bf16(dy2, wf, acc=gres.view(-1, C)) if nat else gres.view(-1, C).addmm_(dy2, wf)
                else:
                    dcol = native.C().mm_bf16(dy2, wf) if nat else torch.mm(dy2, wf)  # [M, Kp]
                    if gres is not None:
                        dcol = dcol + gres.reshape(dcol.shape)
                dx = dcol.view(B, H, W, C) if direct else native.C().col2im_nhwc(dcol, B, H, W, C, R, S, stride, pad)
        return dx, dw, None, None, None


def conv_nhwc(x: torch.Tensor, conv: nn.Conv2d, grad_box: Optional[dict] = None) -> torch.Tensor:
    """``conv(x)`` for a bias-free, ungrouped, undilated Conv2d on a [B, H, W, C] tensor;
    ``grad_box``: the box of a ResidualGradSink on the same input (plain 1x1 convs take its
    gradient into their data-gradient GEMM)"""
    assert conv.bias is None and conv.groups == 1 and conv.dilation == (1, 1), "conv_nhwc: unsupported Conv2d"
    assert conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1], "conv_nhwc: square stride/pad"
    if not x.is_cuda:
        y = F.conv2d(x.permute(0, 3, 1, 2), conv.weight.to(x.dtype), None, conv.stride, conv.padding)
        return y.permute(0, 2, 3, 1).contiguous()
    Co, Ci, R, S = conv.weight.shape
    st, pad = int(conv.stride[0]), int(conv.padding[0])
    # the implicit kernels address every operand with 32-bit buffer offsets (cs_conv_nhwc rejects
    # a tensor of 2 GiB or more): larger convs take the batch-chunked im2col path
    Ho, Wo = (x.shape[1] + 2 * pad - R) // st + 1, (x.shape[2] + 2 * pad - S) // st + 1
    fits = 2 * max(x.numel(), x.shape[0] * Ho * Wo * Co, Co * R * S * max(Ci, 4)) < 0x7ffffff0
    if fits and _implicit_ok(act_dtype(x), x.shape[3], Ci, Co, R, S, st, pad):
        return _ConvImplicitNHWC.apply(x.to(torch.bfloat16).contiguous(), conv.weight, st, pad)
    if fits and _stem_ok(x, Ci, Co, S):
        return _ConvStemNHWC.apply(x.to(torch.bfloat16).contiguous(), conv.weight, st, pad)
    out = _ConvNHWC.apply(x, conv.weight, st, pad, grad_box)
    if isinstance(out, tuple):
        y, tiles = out
        y._cs_bn_tiles = tiles  # read by the bn_act_nhwc on this output
        return y
    return out


def residual_sink_ok(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """whether the block input x can hand its residual gradient to the plain 1x1 ``conv`` on it"""
    return (x.is_cuda and x.requires_grad and torch.is_grad_enabled() and os.environ.get("CS_RES_SINK", "1") != "0"
            and tuple(conv.kernel_size) == (1, 1) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (0, 0))


class _BnActNHWC(torch.autograd.Function):
    """relu(bn(x) + residual): with a residual and ReLU the forward also writes the ReLU mask (one
    bit per element), and the backward's two passes read it instead of the residual to rebuild the
    mask (CS_BN_MASK=0: recompute from x and the residual)"""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu, tiles=None):
        use_mask = relu and residual is not None and os.environ.get("CS_BN_MASK", "1") != "0"
        y, stat, mask = native.C().bn_nhwc_fwd(x, residual, weight, bias, running_mean, running_var, nbt, momentum,
                                               eps, relu, use_mask, tiles)
        ctx.save_for_backward(x, None if use_mask else residual, weight, stat, mask if use_mask else None)
        ctx.relu = relu
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, residual, weight, stat, mask = ctx.saved_tensors
        dx, dres, dw, db = native.C().bn_nhwc_bwd(dy.contiguous(), x, residual, weight, stat, ctx.relu, ctx.has_res,
                                                  mask)
        return (dx, dw, db, dres if ctx.has_res else None, None, None, None, None, None, None, None)


def bn_act_nhwc(bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool = True,
                residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``relu(bn(x) + residual)`` on [B, H, W, C] activations"""
    if (bn.training and bn.track_running_stats and bn.momentum is not None and bn.affine and x.is_cuda
            and x.dtype in (torch.float32, torch.bfloat16) and x.shape[0] * x.shape[1] * x.shape[2] > 1):
        if residual is not None:
            residual = residual.contiguous()
        tiles = getattr(x, "_cs_bn_tiles", None)  # statistics from the producing GEMM, if any
        return _BnActNHWC.apply(x.contiguous(), bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                                bn.num_batches_tracked, float(bn.momentum), float(bn.eps), relu, tiles)
    if bn.training:  # CPU training: the module itself on an NCHW view
        y = bn(x.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    else:
        scale = bn.weight * torch.rsqrt(bn.running_var + bn.eps)
        y = x * scale.to(x.dtype) + (bn.bias - bn.running_mean * scale).to(x.dtype)
    if residual is not None:
        y = y + residual
    return (F.relu(y) if relu else y).contiguous()


class _BnReluPoolNHWC(torch.autograd.Function):
    """max_pool3s2(relu(bn(x))) with the BatchNorm apply fused into the pool's window loads: the
    full-resolution activation is never written (forward) — the ResNet stem's 112x112x64 one is
    411 MB at B=256. Backward: the pool's gather pass, then the BatchNorm backward with the ReLU mask
    recomputed from x (the gather inside both BatchNorm passes measured 0.2-0.4 % slower,
    profiles/r3_resnet50_fusions_ab.txt, and was dropped in round 4)."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, eps):
        y, pos, stat = native.C().bn_relu_maxpool_nhwc_fwd(x, weight, bias, running_mean, running_var, nbt, momentum,
                                                           eps)
        ctx.save_for_backward(x, weight, stat, pos)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, stat, pos = ctx.saved_tensors
        g = native.C().maxpool3s2_nhwc_bwd(dy.contiguous(), pos, x.shape[1], x.shape[2])
        dx, _, dw, db = native.C().bn_nhwc_bwd(g, x, None, weight, stat, True, False)
        return dx, dw, db, None, None, None, None, None


def bn_relu_maxpool_nhwc(bn: nn.BatchNorm2d, x: torch.Tensor) -> torch.Tensor:
    """``max_pool3s2(relu(bn(x)))`` on [B, H, W, C] activations (one fused op in training on the GPU;
    CS_BN_POOL_FUSE=0: BN-apply and pool as two passes)"""
    if (bn.training and bn.track_running_stats and bn.momentum is not None and bn.affine and x.is_cuda
            and x.dtype in (torch.float32, torch.bfloat16) and x.shape[0] * x.shape[1] * x.shape[2] > 1
            and os.environ.get("CS_BN_POOL_FUSE", "1") != "0"):
        return _BnReluPoolNHWC.apply(x.contiguous(), bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                     bn.num_batches_tracked, float(bn.momentum), float(bn.eps))
    return max_pool3s2_nhwc(bn_act_nhwc(bn, x))


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, pos = native.C().maxpool3s2_nhwc_fwd(x)
        ctx.save_for_backward(pos)
        ctx.hw = (x.shape[1], x.shape[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        (pos,) = ctx.saved_tensors
        return native.C().maxpool3s2_nhwc_bwd(dy.contiguous(), pos, *ctx.hw)


def max_pool3s2_nhwc(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(., 3, 2, 1)`` on a [B, H, W, C] tensor"""
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16):
        return _MaxPoolNHWC.apply(x.contiguous())
    return F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).contiguous()
