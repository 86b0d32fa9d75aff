"""Fused training BatchNorm2d (+ residual add) (+ ReLU) for NCHW activations
(``csrc/kernels/bn_nchw.hip``), used by the ResNet models in place of
``relu(bn(x) + residual)``.

``bn_act(bn, x, relu, residual)`` runs the gfx950 kernels when ``bn`` is training with batch
statistics and running stats (momentum not None), and ``x`` is a contiguous NCHW fp32 / bf16
GPU tensor: one statistics pass, one normalise/add/ReLU pass, and in the backward one reduction
pass and one dx (+ residual gradient) pass, with the ReLU mask recomputed from the saved input
instead of stored. Running mean / var and ``num_batches_tracked`` are updated like
``nn.BatchNorm2d``, inside the statistics launch. Anything else (CPU, eval mode, channels_last) runs the module itself.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import native


class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, momentum, eps, relu):
        y, stat = native.C().bn_act_fwd(x, residual, weight, bias, running_mean, running_var, nbt, momentum, eps,
                                        relu)
        ctx.save_for_backward(x, residual, weight, stat)
        ctx.relu = relu
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, residual, weight, stat = ctx.saved_tensors
        dx, dres, dw, db = native.C().bn_act_bwd(dy.contiguous(), x, residual, weight, stat, ctx.relu, ctx.has_res)
        return (dx, dw if weight is not None else None, db if weight is not None else None,
                dres if ctx.has_res else None, None, None, None, None, None, None)


def native_ok(bn: nn.BatchNorm2d, x: torch.Tensor, residual: Optional[torch.Tensor]) -> bool:
    return (bn.training and bn.track_running_stats and bn.momentum is not None and bn.affine
            and x.is_cuda and x.dim() == 4 and x.is_contiguous() and x.dtype in (torch.float32, torch.bfloat16)
            and x.shape[0] * x.shape[2] * x.shape[3] > 1
            and (residual is None or (residual.shape == x.shape and residual.dtype == x.dtype)))


def bn_act(bn: nn.BatchNorm2d, x: torch.Tensor, relu: bool = True,
           residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    if native_ok(bn, x, residual):
        if residual is not None:
            residual = residual.contiguous()
        return _BnAct.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                            bn.num_batches_tracked, float(bn.momentum), float(bn.eps), relu)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y, pos = native.C().maxpool3s2_fwd(x)
        ctx.save_for_backward(pos)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        (pos,) = ctx.saved_tensors
        return native.C().maxpool3s2_bwd(dy.contiguous(), pos, *ctx.hw)


def max_pool3s2(x: torch.Tensor) -> torch.Tensor:
    """``F.max_pool2d(x, 3, 2, 1)``: the gfx950 kernels for contiguous NCHW fp32 / bf16 GPU
    tensors (gather-style deterministic backward), ATen otherwise."""
    if x.is_cuda and x.dim() == 4 and x.is_contiguous() and x.dtype in (torch.float32, torch.bfloat16):
        return _MaxPool3s2.apply(x)
    return F.max_pool2d(x, 3, 2, 1)
