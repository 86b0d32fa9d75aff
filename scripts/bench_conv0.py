"""Isolated timing of the direct VGG block-0 kernels (csrc/kernels/conv0.hip) at the bench shape.

    python scripts/bench_conv0.py [--batch 64] [--iters 200]

Prints one JSON line: microseconds per call of conv0_fwd (with BN tile statistics), conv0_fwd
without statistics and conv0_wgrad (partials + fixed-order sum), plus the traffic-bound floor of
each at 8 TB/s. Needs a GPU.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    dev = "cuda"
    B = args.batch
    x = torch.randn(B, 32, 32, 4, device=dev)
    w = torch.randn(64, 3, 3, 3, device=dev)
    bias = torch.randn(64, device=dev)
    dz = torch.randn(B * 1024, 64, device=dev)
    fwd = _time(lambda: C.conv0_fwd(x, w, bias, True), args.iters)
    fwd_ns = _time(lambda: C.conv0_fwd(x, w, bias, False), args.iters)
    wg = _time(lambda: C.conv0_wgrad(x, dz), args.iters)
    ybytes = B * 1024 * 64 * 4
    print(json.dumps({"batch": B, "fwd_stats_us": round(fwd, 2), "fwd_us": round(fwd_ns, 2),
                      "wgrad_us": round(wg, 2), "floor_fwd_us": round(ybytes / 8e12 * 1e6, 2),
                      "floor_wgrad_us": round(ybytes / 8e12 * 1e6, 2)}))


if __name__ == "__main__":
    main()
