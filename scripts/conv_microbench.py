"""Conv implicit-GEMM microbenchmark: TFLOP/s of each tile config at a small (B=64) and a
large (B=512) batch, fwd/dgrad/wgrad of a VGG-11 layer; separates core-loop efficiency
from small-problem (ramp / tail / split-K) effects."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn

dev = torch.device("cuda", 0)
out = []


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


SHAPES = [(64, 8, 256, 256), (512, 8, 256, 256), (64, 4, 512, 512), (256, 4, 512, 512), (64, 16, 64, 128)]
if os.environ.get("MICRO_SHAPES"):
    SHAPES = [SHAPES[int(i)] for i in os.environ["MICRO_SHAPES"].split(",")]
for B, H, cin, cout in SHAPES:
    x = torch.randn(B, H, H, cin, device=dev)
    w = torch.randn(cout, 3, 3, cin, device=dev) * 0.05
    bias = torch.zeros(cout, device=dev)
    dz = torch.randn(B * H * H, cout, device=dev)
    flops = 2.0 * B * H * H * cout * cin * 9
    best = {}
    for bm, bn in [(64, 64), (128, 64), (64, 128), (128, 128)]:
        for bk in (16, 32):
            for sp in (1, 2, 4, 8, 16):
                for mode in ("fwd", "dgrad", "wgrad"):
                    if mode == "fwd":
                        f = lambda: Fn.conv_fwd(x, w, bias, bm=bm, bn=bn, splits=sp, bk=bk, stats=True)
                    elif mode == "dgrad":
                        f = lambda: Fn.conv_dgrad(dz, w, B, H, H, bm=bm, bn=bn, splits=sp, bk=bk)
                    else:
                        f = lambda: Fn.conv_wgrad(dz, x, cout, bm=bm, bn=bn, splits=sp, bk=bk)
                    us = timeit(f)
                    tf = flops / us / 1e6
                    key = mode
                    if key not in best or tf > best[key][0]:
                        best[key] = (tf, us, bm, bn, bk, sp)
    for mode, (tf, us, bm, bn, bk, sp) in best.items():
        row = dict(sched=os.environ.get("CS_CONV_SCHED", "0"), B=B, H=H, cin=cin, cout=cout, mode=mode, tflops=round(tf, 1), us=round(us, 2), bm=bm, bn=bn,
                   bk=bk, splits=sp)
        print(json.dumps(row), flush=True)
