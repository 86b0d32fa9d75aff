"""XP K-loop ablation (CS_XP_PROBE, wrong numbers): graph-timed fwd GEMM of VGG-11 block 3
(M 4096, N 256, K 2304) and block 5 (M 1024, N 512, K 4608) at 64x64/bk64/kg2 and
128x128/bk32/kg2 with the full loop, no in-loop DMA, no MFMA, DMA only."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1:  # child: one probe mode (the env var is read once per process)
    sys.path.insert(0, ROOT)
    import torch
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    sys.argv = sys.argv[:1] + ["64", "10"]
    C = native.C()
    dev = torch.device("cuda", 0)
    WS = torch.empty(16 << 20, device=dev)
    B = 64
    out = {}
    for l, (H, cin, cout) in ((3, (8, 256, 256)), (5, (4, 512, 512))):
        x3 = Fn.split3(torch.randn(B, H, H, cin, device=dev))
        w3 = Fn.split3(torch.randn(cout, 3, 3, cin, device=dev) * 0.05)
        y = torch.empty(B * H * H * cout, device=dev)
        for (bm, bk, sp) in ((64, 64, 1 if l == 3 else 2), (128, 32, 4 if l == 3 else 8)):
            f = lambda: C.conv_gemm_xp(0, x3, w3, None, None, y, WS, None, B, H, H, cin, cout, bm, bm, sp, bk, 2, 0)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    f()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[f"b{l}_{bm}x{bm}_bk{bk}_s{sp}"] = round(e0.elapsed_time(e1) / 100 * 1e3, 2)
    print(json.dumps(out))
    sys.exit(0)
for p in ("0", "1", "2", "3"):
    env = dict(os.environ, CS_XP_PROBE=p)
    r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    print(json.dumps({"probe": {"0": "full", "1": "no_dma", "2": "no_mfma", "3": "dma_only"}[p],
                      "us": json.loads(line[-1]) if line else r.stderr[-400:]}), flush=True)
