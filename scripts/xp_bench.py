"""Pre-split ("XP") conv GEMM sweep on the VGG-11 training shapes vs the shipped tuned
kernels (runtime/tiles_gfx950.json), both timed as graph-captured launches (no Python
launch overhead in the numbers). Usage: python scripts/xp_bench.py [B] [reps] [only_block]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn  # noqa: E402
from cs744_pytorch_distributed_tutorial_amd.ops import native  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ONLY = int(sys.argv[3]) if len(sys.argv) > 3 else -1
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
C = native.C()
BLOCKS = [(16, 64, 128), (8, 128, 256), (8, 256, 256), (4, 256, 512), (4, 512, 512), (2, 512, 512), (2, 512, 512)]
TILES = [(bm, bn, bk, kg, nb) for bm in (64, 128) for bn in (64, 128) for bk in (32, 64) for kg in (1, 2)
         for nb in range(4) if C.conv_xp_ok(bm, bn, bk, kg, nb)]
SPLITS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
table = json.load(open(os.path.join(ROOT, "cs744_pytorch_distributed_tutorial_amd", "runtime", "tiles_gfx950.json")))
entry = table.get(f"VGG11/B{B}/gfx950/v2", {})
tuned = {(t[0], t[1]): t[2:] for t in entry.get("tiles", [])}  # (block, mode) -> bm, bn, splits, bk, stage
WS = torch.empty(16 << 20, device=dev)


def gtime(fn, n=10):
    """us per call: n calls captured in one graph, replayed REPS times."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (REPS * n) * 1e3


tot_xp = tot_ref = tot_min = 0.0
for l, (H, cin, cout) in enumerate(BLOCKS, start=1):
    if ONLY >= 0 and l != ONLY:
        continue
    x = torch.randn(B, H, H, cin, device=dev)
    w = torch.randn(cout, 3, 3, cin, device=dev) * 0.05
    dz = torch.randn(B * H * H, cout, device=dev)
    bias = torch.zeros(cout, device=dev)
    x3, w3, dz3 = Fn.split3(x), Fn.split3(w), Fn.split3(dz)
    for mode, name in ((0, "fwd"), (1, "dgrad"), (2, "wgrad")):
        M, N, K = Fn.gemm_dims(mode, B, H, H, cin, cout)
        out = torch.empty(max(M * N, cout * 9 * cin), device=dev)
        stats = torch.empty(((M + 15) // 16) * N * 2, device=dev)
        best = None
        for (bm, bn, bk, kg, nb) in TILES:
            for sp in SPLITS:
                if sp > 1 and K // bk < 2 * sp:
                    continue
                if sp * M * N > WS.numel():
                    continue
                f = lambda: C.conv_gemm_xp(mode, x3 if mode != 1 else None, w3 if mode != 2 else None,  # noqa
                                           dz3 if mode != 0 else None, bias if mode == 0 else None, out, WS,
                                           stats if mode == 0 else None, B, H, H, cin, cout, bm, bn, sp, bk, kg, nb)
                us = gtime(f)
                if best is None or us < best[0]:
                    best = (us, bm, bn, bk, kg, sp, nb)
        ref = float("nan")
        if (l, mode) in tuned:
            bm, bn, sp, bk, stage = tuned[(l, mode)]
            wt = w.contiguous()
            f = lambda: C.conv_gemm(mode, x if mode != 1 else None, wt if mode != 2 else None,  # noqa
                                    dz if mode != 0 else None, bias if mode == 0 else None, out, WS,
                                    stats if mode == 0 else None, B, H, H, cin, cout, False, bm, bn, sp, bk, None,
                                    stage)
            ref = gtime(f)
        tot_xp += best[0]
        tot_ref += ref
        tot_min += min(best[0], ref)
        tf = 2.0 * M * N * K / best[0] / 1e6
        print(json.dumps(dict(block=l, mode=name, M=M, N=N, K=K, xp_us=round(best[0], 2), tflops=round(tf, 1),
                              ref_us=round(ref, 2), bm=best[1], bn=best[2], bk=best[3], kg=best[4],
                              splits=best[5], nb=best[6])), flush=True)
print(json.dumps(dict(total_xp_us=round(tot_xp, 1), total_ref_us=round(tot_ref, 1), total_min_us=round(tot_min, 1))),
      flush=True)
