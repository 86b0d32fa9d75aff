"""Decoder-only LM with the Llama-3 architecture (BASELINE.json config "Llama-3 8B
bf16 pure data-parallel grad all-reduce on 8xMI355X" — an extension; the
reference has no language model).

Pre-norm blocks: RMSNorm -> grouped-query attention with rotary position
embeddings (RoPE, theta 500000) -> residual -> RMSNorm -> SwiGLU MLP -> residual;
untied input embedding / output head. Pure data parallelism: every rank holds
the full replica (8.03 B parameters = 16 GB in bf16, fits the 288 GB HBM3E of one
MI355X with gradients and optimizer state), and the step's 16 GB of bf16
gradients is the xGMI all-reduce stress the config names.

Hot ops have hand-written gfx950 kernels used on the GPU: RMSNorm fwd/bwd, SwiGLU
fwd/bwd and RoPE in ``ops.lm``, and causal grouped-query flash attention (forward and a
deterministic backward, bf16, head dim 64/128) in ``ops.attention`` — called on the
[B, S, H, D] projections directly, no transposes. The projection GEMMs are plain library
GEMMs (hipBLASLt), run on bf16 copies of the fp32 master weights that the fused SGD pass
rewrites (``ops.lm.ShadowLinear``): no per-step weight casts, fp32 weight gradients straight out
of the GEMM.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    vocab_size: int = 128256
    max_seq: int = 8192
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5


CONFIGS = {
    "llama3-8b": LlamaConfig(),
    "llama3-1b": LlamaConfig(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192, max_seq=2048),
    "llama-tiny": LlamaConfig(dim=256, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=512, vocab_size=1024,
                              max_seq=128),
}


def _ops():
    from ..ops import lm
    return lm


def _Linear(*args, **kwargs) -> nn.Linear:
    """bias-free projection: ``ops.lm.ShadowLinear`` (nn.Linear with a bf16 weight copy kept in step
    with the fp32 master by the fused optimizer)"""
    from ..ops.lm import ShadowLinear
    return ShadowLinear(*args, **kwargs)


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _ops().rms_norm(x, self.weight, self.eps)


def rope_tables(seq: int, head_dim: int, theta: float, device) -> tuple:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, device=device, dtype=torch.float32) / head_dim))
    ang = torch.outer(torch.arange(seq, device=device, dtype=torch.float32), inv)
    return ang.cos(), ang.sin()


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.nh, self.nkv = cfg.n_heads, cfg.n_kv_heads
        self.hd = cfg.dim // cfg.n_heads
        self.wq = _Linear(cfg.dim, self.nh * self.hd, bias=False)
        self.wk = _Linear(cfg.dim, self.nkv * self.hd, bias=False)
        self.wv = _Linear(cfg.dim, self.nkv * self.hd, bias=False)
        self.wo = _Linear(self.nh * self.hd, cfg.dim, bias=False)

    def forward(self, x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
        B, S, _ = x.shape
        q = self.wq(x).view(B, S, self.nh, self.hd)
        k = self.wk(x).view(B, S, self.nkv, self.hd)
        v = self.wv(x).view(B, S, self.nkv, self.hd)
        q, k = _ops().rope(q, cos, sin), _ops().rope(k, cos, sin)
        from ..ops.attention import attention, native_ok
        if native_ok(q, k, v):
            o = attention(q, k, v, causal=True)  # [B, S, Hq, hd], gfx950 flash attention
        else:  # CPU / fp32: PyTorch's attention
            q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=self.nkv != self.nh).transpose(1, 2)
        return self.wo(o.reshape(B, S, self.nh * self.hd))


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w1 = _Linear(cfg.dim, cfg.ffn_dim, bias=False)  # gate
        self.w3 = _Linear(cfg.dim, cfg.ffn_dim, bias=False)  # up
        self.w2 = _Linear(cfg.ffn_dim, cfg.dim, bias=False)  # down

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.w2(_ops().swiglu(self.w1(x), self.w3(x)))


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attention_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x, cos, sin):
        x = x + self.attention(self.attention_norm(x), cos, sin)
        return x + self.feed_forward(self.ffn_norm(x))


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.vocab_size, self.max_seq = cfg.vocab_size, cfg.max_seq
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList(Block(cfg) for _ in range(cfg.n_layers))
        self.norm = RMSNorm(cfg.dim, cfg.norm_eps)
        self.output = _Linear(cfg.dim, cfg.vocab_size, bias=False)
        std = 0.02
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, std)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, 0.0, std)
        for blk in self.layers:  # scaled residual projections
            nn.init.normal_(blk.attention.wo.weight, 0.0, std / math.sqrt(2 * cfg.n_layers))
            nn.init.normal_(blk.feed_forward.w2.weight, 0.0, std / math.sqrt(2 * cfg.n_layers))
        self._rope = None

    def _tables(self, S: int, device):
        if self._rope is None or self._rope[0].shape[0] < S or self._rope[0].device != device:
            self._rope = rope_tables(max(S, 1), self.cfg.dim // self.cfg.n_heads, self.cfg.rope_theta, device)
        return self._rope[0][:S], self._rope[1][:S]

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        S = tokens.shape[1]
        cos, sin = self._tables(S, tokens.device)
        h = self.tok_embeddings(tokens)
        for blk in self.layers:
            h = blk(h, cos, sin)
        return self.output(self.norm(h))


def build(name: str) -> Llama:
    key = name.lower().replace("_", "-")
    if key in ("llama3-8b", "llama-3-8b", "llama38b"):
        key = "llama3-8b"
    if key not in CONFIGS:
        raise ValueError(f"unknown LM config {name!r}; choose from {sorted(CONFIGS)}")
    return Llama(CONFIGS[key])


def param_count(cfg: LlamaConfig) -> int:
    hd = cfg.dim // cfg.n_heads
    attn = cfg.dim * hd * (cfg.n_heads * 2 + cfg.n_kv_heads * 2)
    ffn = 3 * cfg.dim * cfg.ffn_dim
    return cfg.n_layers * (attn + ffn + 2 * cfg.dim) + 2 * cfg.vocab_size * cfg.dim + cfg.dim
