"""bf16 GEMM shapes of the Llama-3-8B projections (8 x 2048 tokens): the gemm_bf16.hip kernel vs
torch.mm (hipBLASLt) on the same uniform [-1, 1) operands, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rules 24/25), for all three products of each projection (forward,
data gradient, fp32 weight gradient). One JSON line per product: median / best TF of each.

Usage (GPU box): python scripts/gemm_bench.py [--tokens 16384] [--rounds 5] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

# (name, N, K): y[tokens, N] = x[tokens, K] . W[N, K]^T
SHAPES = [
    ("wq/wo", 4096, 4096),
    ("wk/wv", 1024, 4096),
    ("w1/w3", 14336, 4096),
    ("w2", 4096, 14336),
    ("lm_head", 128256, 4096),
]


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tokens", type=int, default=16384)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--shapes", type=str, default="")
    p.add_argument("--products", type=str, default="")
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, N, K in SHAPES:
        if a.shapes and name not in a.shapes.split(","):
            continue
        M = a.tokens
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        dy = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).bfloat16()
        # the three products of the projection: (label, ours, hipBLASLt)
        prods = [
            ("y=xW^T", lambda: C.mm_bf16(x, w.t()), lambda: torch.mm(x, w.t())),
            ("dx=dyW", lambda: C.mm_bf16(dy, w), lambda: torch.mm(dy, w)),
            ("dW=dy^Tx", lambda: C.mm_bf16(dy.t(), x, True), lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)),
        ]
        flop = 2.0 * M * N * K
        for label, ours, blas in prods:
            if a.products and label not in a.products.split(","):
                continue
            y0, y1 = ours(), blas()
            err = ((y0.float() - y1.float()).abs().max() / y1.float().abs().max()).item()
            del y0, y1
            t = {"ours": [], "hipblaslt": []}
            for _ in range(a.rounds):
                for k, fn in (("ours", ours), ("hipblaslt", blas)):
                    fn()
                    t[k].append(timed(fn, a.reps))
            row = {"shape": name, "product": label, "M": M, "N": N, "K": K, "max_rel_diff": round(err, 5)}
            for k, v in t.items():
                row[f"{k}_ms_med"] = round(statistics.median(v), 4)
                row[f"{k}_tflops_med"] = round(flop / statistics.median(v) / 1e9, 1)
                row[f"{k}_tflops_best"] = round(flop / min(v) / 1e9, 1)
            row["ours_vs_hipblaslt"] = round(statistics.median(t["hipblaslt"]) / statistics.median(t["ours"]), 3)
            print(json.dumps(row), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
