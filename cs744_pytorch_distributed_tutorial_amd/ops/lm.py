"""Autograd wrappers of the decoder-LM gfx950 kernels (``csrc/kernels/lm.hip``).

On GPU tensors every op runs the hand-written HIP kernel (forward and backward);
on CPU tensors the plain-PyTorch reference below runs instead (this is the
numerics oracle of ``tests/test_lm_gpu.py`` and lets the LM train on CPU in the
multi-process gloo tests).
"""
from __future__ import annotations

import os

import torch

from . import native


# ------------------------------------------------------------------ references
def rms_norm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def swiglu_ref(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return (torch.nn.functional.silu(a.float()) * b.float()).to(a.dtype)


def rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, S, H, hd], rotate interleaved pairs (2j, 2j+1) by angle table [S, hd/2]."""
    xf = x.float().view(*x.shape[:-1], -1, 2)
    c = cos[None, :, None, :]
    s = sin[None, :, None, :]
    x0, x1 = xf[..., 0], xf[..., 1]
    out = torch.stack([x0 * c - x1 * s, x0 * s + x1 * c], -1)
    return out.view(x.shape).to(x.dtype)


# ------------------------------------------------------------------ autograd functions
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, out_bf16):
        xc = x.contiguous()
        y, rstd = native.C().rmsnorm_fwd(xc, w.contiguous(), eps, out_bf16)
        ctx.save_for_backward(xc, w, rstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, rstd = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != x.dtype and x.shape[-1] % 4 != 0:
            gy = gy.to(x.dtype)
        dx, dw = native.C().rmsnorm_bwd(x, w.contiguous(), rstd, gy)
        return dx, dw, None, None


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        ctx.save_for_backward(a, b)
        return native.C().swiglu_fwd(a, b)

    @staticmethod
    def backward(ctx, gy):
        a, b = ctx.saved_tensors
        da, db = native.C().swiglu_bwd(a, b, gy.contiguous().to(a.dtype))
        return da, db


class _RoPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        cos, sin = cos.float().contiguous(), sin.float().contiguous()
        ctx.save_for_backward(cos, sin)
        return native.C().rope(x.contiguous(), cos, sin, False)

    @staticmethod
    def backward(ctx, gy):
        cos, sin = ctx.saved_tensors
        return native.C().rope(gy.contiguous(), cos, sin, True), None, None


def _native_ok(*ts) -> bool:
    return all(t.is_cuda for t in ts) and all(t.dtype in (torch.float32, torch.bfloat16) for t in ts)


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if _native_ok(x, w):
        # under bf16 autocast the fp32 residual stream is normalised straight into bf16: the
        # projections that follow read it without a cast pass each (5 per block), and their input
        # gradients come back in bf16 into the backward kernel, again without a cast
        out_bf16 = (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
                    and x.shape[-1] % 4 == 0)
        return _RMSNorm.apply(x, w, eps, out_bf16)
    return rms_norm_ref(x, w, eps)


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if _native_ok(a, b) and a.dtype == b.dtype:
        return _SwiGLU.apply(a, b)
    return swiglu_ref(a, b)


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    if _native_ok(x):
        return _RoPE.apply(x, cos, sin)
    return rope_ref(x, cos, sin)


# ------------------------------------------------------------------ bf16 projections with fp32 masters
# "native": the gfx950 matrix-core GEMM of csrc/kernels/gemm_bf16.hip runs all three products of a
# projection (y = x W^T, dx = dy W, dW = dy^T x, the last two reading the operands transposed in
# LDS, no copies); "wgrad": it runs the fp32 weight gradient dW only (where it measured faster
# than hipBLASLt at every Llama-3-8B shape, profiles/r4_gemm_bench_v2.jsonl); "blas": torch.mm
# (hipBLASLt) for all three. scripts/gemm_bench.py compares them per shape.
_GEMM = os.environ.get("CS_LM_GEMM", "wgrad")
if _GEMM not in ("native", "wgrad", "blas"):
    raise ValueError(f"CS_LM_GEMM must be 'native', 'wgrad' or 'blas', got {_GEMM!r}")


def gemm_operands_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Whether ``native.C().mm_bf16(a, b)`` can run ``a @ b`` in place: the host-side preconditions
    of ``cs_gemm_bf16`` (csrc/kernels/gemm_bf16.hip), checked here so an operand the kernel cannot
    read (no unit stride — e.g. an expanded stride-0 gradient —, a leading dimension or an N that is
    not a multiple of 8 / 4 — an odd vocabulary —, a base pointer off 16 bytes) goes to torch.mm
    instead of raising inside backward."""
    if a.dim() != 2 or b.dim() != 2 or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda:
        return False
    M, K = a.shape
    N = b.shape[1]
    if M == 0 or N == 0 or K == 0:
        return True  # mm_bf16 returns zeros without a launch
    if a.stride(1) == 1:
        a_kmajor, lda = True, a.stride(0)
    elif a.stride(0) == 1:
        a_kmajor, lda = False, a.stride(1)
    else:
        return False
    if b.stride(0) == 1:
        b_kmajor, ldb = True, b.stride(1)
    elif b.stride(1) == 1:
        b_kmajor, ldb = False, b.stride(0)
    else:
        return False
    if lda % 8 or ldb % 8 or N % 4:
        return False
    if (a_kmajor or b_kmajor) and K % 8:
        return False
    if (lda < K if a_kmajor else lda < M) or (ldb < K if b_kmajor else ldb < N):
        return False
    # 32-bit buffer offsets: a K-major operand addresses 256 rows (kTile), an M-major one 64 k rows
    # (kBK) per tile; and the tile count fits an int (cs_gemm_bf16's own checks, mirrored)
    if (256 if a_kmajor else 64) * lda * 2 >= 0x7fffffff or (256 if b_kmajor else 64) * ldb * 2 >= 0x7fffffff:
        return False
    if ((M + 255) // 256) * ((N + 255) // 256) > 0x7fffffff:
        return False
    return (a.data_ptr() | b.data_ptr()) % 16 == 0


def _mm(a: torch.Tensor, b: torch.Tensor, out_f32: bool = False) -> torch.Tensor:
    """a @ b for bf16 2-D operands (views allowed), bf16 or fp32 out (fp32: the weight gradient)"""
    if (_GEMM == "native" or (_GEMM == "wgrad" and out_f32)) and gemm_operands_ok(a, b):
        return native.C().mm_bf16(a, b, out_f32)
    if out_f32:
        return torch.mm(a, b, out_dtype=torch.float32)
    return torch.mm(a, b)


class _LinearShadow(torch.autograd.Function):
    """y = x @ W^T on the bf16 shadow of the fp32 master W; dW straight out of the GEMM in fp32"""

    @staticmethod
    def forward(ctx, x, weight, shadow):
        x2 = x.reshape(-1, x.shape[-1])
        with torch.autocast("cuda", enabled=False):
            y = _mm(x2, shadow.t())
        ctx.save_for_backward(x2, shadow)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], shadow.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, shadow = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1])
        if g2.dtype != shadow.dtype:
            g2 = g2.to(shadow.dtype)
        dx = dw = None
        with torch.autocast("cuda", enabled=False):
            if ctx.needs_input_grad[0]:
                dx = _mm(g2, shadow).view(ctx.xshape)
            if ctx.needs_input_grad[1]:
                dw = _mm(g2.t(), x2, out_f32=True)
        return dx, dw, None


class ShadowLinear(torch.nn.Linear):
    """``nn.Linear`` (same parameters and state_dict) whose bf16-autocast forward reads a bf16 copy
    of the fp32 weight kept alongside it instead of casting the weight at every use. ``FusedSGD``
    rewrites the copy in its update pass (``sgd_multi`` shadow column), so a training step spends no
    cast kernel on the weights at all, and the weight gradient leaves the GEMM in fp32 (no bf16
    round trip, no cast back). Any other in-place change of the weight (load_state_dict, a DDP
    broadcast, another optimizer) bumps its version and the copy is re-made on the next forward."""

    def _shadow(self) -> torch.Tensor:
        w = self.weight
        sh = getattr(w, "_cs_bf16_shadow", None)
        if sh is None or getattr(w, "_cs_bf16_shadow_version", -1) != w._version or sh.device != w.device \
                or sh.shape != w.shape:
            with torch.no_grad():
                sh = w.detach().to(torch.bfloat16)
            w._cs_bf16_shadow = sh
            w._cs_bf16_shadow_version = w._version
        return sh

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (self.bias is None and x.is_cuda and self.weight.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return _LinearShadow.apply(x.to(torch.bfloat16), self.weight, self._shadow())
        return super().forward(x)


# ------------------------------------------------------------------ LM loss
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets):
        loss, lse = native.C().xent_fwd(logits, targets)
        ctx.save_for_backward(logits, targets, lse)
        return loss.sum() / logits.shape[0]

    @staticmethod
    def backward(ctx, g):
        logits, targets, lse = ctx.saved_tensors
        d = native.C().xent_bwd(logits, targets, lse, g.float().reshape(1).contiguous(), 1.0 / logits.shape[0])
        return d, None


def cross_entropy(logits: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
    """``F.cross_entropy(logits.float(), targets)`` (mean over rows) for [R, V] logits: on GPU one
    fused gfx950 pass forward and one backward over the logits in their own dtype (no fp32 upcast of
    the [tokens, vocab] matrix, no separate log-softmax / nll / cast kernels). Targets must lie in
    [0, V) (no ignore index; the LM's synthetic tokens always do)."""
    if (logits.is_cuda and logits.dim() == 2 and logits.shape[1] % 8 == 0
            and logits.dtype in (torch.float32, torch.bfloat16)):
        return _CrossEntropy.apply(logits.contiguous(), targets.contiguous())
    return torch.nn.functional.cross_entropy(logits.float(), targets)
