"""Grouped-query flash attention on gfx950 (``csrc/kernels/attention.hip``) as an autograd op.

``attention(q, k, v, causal)`` takes the Llama model's natural layout — q ``[B, S, Hq, D]``,
k/v ``[B, S, Hkv, D]`` — and returns ``[B, S, Hq, D]``. bf16 GPU tensors with D in {64, 128}
run the native forward (online softmax, row log-sum-exp kept for the backward) and the
deterministic native backward (delta, dQ per query block, dK/dV per key block over the
whole query-head group). Anything else — CPU tensors (the gloo tests), fp32, other head
sizes — runs the plain-PyTorch reference below, which is also the numerics oracle of
``tests/test_attention_gpu.py``.
"""
from __future__ import annotations

import math

import torch

from . import native


def attention_ref(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True) -> torch.Tensor:
    """Math attention in fp32 on [B, S, H, D] tensors (GQA by head repetition)."""
    B, S, Hq, D = q.shape
    rep = Hq // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().repeat_interleave(rep, dim=2).transpose(1, 2)
    vf = v.float().repeat_interleave(rep, dim=2).transpose(1, 2)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    o = torch.softmax(s, -1) @ vf
    return o.transpose(1, 2).to(q.dtype)


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        scale = 1.0 / math.sqrt(q.shape[-1])
        o, lse = native.C().attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = native.C().attn_bwd(q, k, v, o, lse, do.contiguous().to(q.dtype), ctx.scale, ctx.causal)
        return dq, dk, dv, None


def native_ok(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> bool:
    return (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype
            and q.shape[-1] in (64, 128) and q.shape[2] % k.shape[2] == 0)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True) -> torch.Tensor:
    if native_ok(q, k, v):
        return _FlashAttention.apply(q, k, v, causal)
    return attention_ref(q, k, v, causal)
