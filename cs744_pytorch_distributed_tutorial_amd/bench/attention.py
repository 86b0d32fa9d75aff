"""Attention throughput on one GPU: the gfx950 flash attention (ops/attention.py) vs
PyTorch's scaled_dot_product_attention, at the Llama-3 8B attention shape (Hq 32, Hkv 8,
D 128, causal, bf16). FLOPs counted as 4*B*Hq*S*S*D (forward, halved for causal) and 3.5x
that for forward+backward (the backward's five products, 2.5x the forward's two).

    python -m cs744_pytorch_distributed_tutorial_amd.bench.attention --seq 2048 4096
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F


def _time(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main(argv=None) -> None:
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--seq", type=int, nargs="+", default=[2048, 4096])
    p.add_argument("--heads", type=int, default=32)
    p.add_argument("--kv-heads", type=int, default=8)
    p.add_argument("--head-dim", type=int, default=128)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args(argv)
    from ..ops.attention import attention
    dev = torch.device("cuda", 0)
    for S in a.seq:
        B, Hq, Hkv, D = a.batch, a.heads, a.kv_heads, a.head_dim
        q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, S, Hkv, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
        do = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
        flops = 4.0 * B * Hq * S * S * D / 2  # causal

        def ours_f():
            with torch.no_grad():
                attention(q, k, v, True)

        def ours_fb():
            attention(q, k, v, True).backward(do)

        qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
        dot = do.transpose(1, 2).contiguous()

        def sdpa_f():
            with torch.no_grad():
                F.scaled_dot_product_attention(qt, kt, vt, is_causal=True, enable_gqa=True)

        def sdpa_fb():
            F.scaled_dot_product_attention(qt, kt, vt, is_causal=True, enable_gqa=True).backward(dot)

        row = {"B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "D": D}
        for name, fn, fl in (("native_fwd", ours_f, flops), ("native_fwd_bwd", ours_fb, 3.5 * flops),
                             ("sdpa_fwd", sdpa_f, flops), ("sdpa_fwd_bwd", sdpa_fb, 3.5 * flops)):
            try:
                ms = _time(fn, a.iters)
                row[name + "_ms"] = round(ms, 4)
                row[name + "_tflops"] = round(fl / ms / 1e9, 1)
            except RuntimeError as e:  # e.g. an SDPA backend without GQA support
                row[name + "_error"] = str(e)[:120]
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
