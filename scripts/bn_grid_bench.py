"""Graph-timed BN forward/backward variants at the VGG-11 CIFAR shapes (B = 64), one line per layer:
split launches (finalize + apply / reduce + finalize + apply), the single-block fused kernels, and
the one-launch grid-barrier kernels (csrc/kernels/bn_grid.hip). Knobs read by the grid launchers:
CS_BN_GRID_PMUL (blocks per CU for the forward), CS_BN_GRID_BARV (barrier version; -1 = barriers skipped: timing of
the phases alone, results wrong). Usage: python scripts/bn_grid_bench.py [B] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cs744_pytorch_distributed_tutorial_amd.ops import functional as F  # noqa: E402

SHAPES = [(32, 32, 64, True), (16, 16, 128, True), (8, 8, 256, False), (8, 8, 256, True),
          (4, 4, 512, False), (4, 4, 512, True), (2, 2, 512, False), (2, 2, 512, True)]


def graph_us(fn, reps):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (5 * reps)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    print(f"# B={B} PMUL={os.environ.get('CS_BN_GRID_PMUL', '1')} BARV={os.environ.get('CS_BN_GRID_BARV', '2')}")
    print(f"{'H':>3} {'C':>4} pool | fwd split  fused   grid | bwd split  fused   grid   (us per call)")
    for H, W, C, pool in SHAPES:
        M = B * H * W
        rows = 64
        y = torch.randn(M, C, device=dev)
        T = M // rows
        t = y.view(T, rows, C)
        stats = torch.stack([t.mean(1), ((t - t.mean(1, keepdim=True)) ** 2).sum(1)], -1).contiguous()
        gamma = torch.rand(C, device=dev) + 0.5
        beta = torch.randn(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        Ho, Wo = (H // 2, W // 2) if pool else (H, W)
        G = torch.randn(B * Ho * Wo, C, device=dev)
        row = []
        for mode in (False, True, "grid"):
            try:
                row.append(graph_us(lambda: F.bn_relu_pool_fwd(y, stats, rows, B, H, W, gamma, beta, rm, rv, nbt,
                                                               pool=pool, fused=mode), reps))
            except Exception as e:  # a variant that does not serve this shape
                print("#", mode, type(e).__name__, str(e)[:80])
                row.append(float("nan"))
        _, st = F.bn_relu_pool_fwd(y, stats, rows, B, H, W, gamma, beta, pool=pool)
        for mode in (False, True, "grid"):
            try:
                row.append(graph_us(lambda: F.bn_relu_pool_bwd(y, G, st, gamma, B, H, W, pool=pool, fused=mode), reps))
            except Exception as e:
                print("#", mode, type(e).__name__, str(e)[:80])
                row.append(float("nan"))
        print(f"{H:>3} {C:>4} {int(pool):>4} | " + " ".join(f"{v:7.2f}" for v in row[:3]) + " | "
              + " ".join(f"{v:7.2f}" for v in row[3:]), flush=True)


if __name__ == "__main__":
    main()
