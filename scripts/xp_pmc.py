"""Drive a few pre-split conv GEMM configs (5 launches each) for rocprofv3 counter passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn  # noqa: E402
from cs744_pytorch_distributed_tutorial_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
C = native.C()
B = 64
BLOCKS = {3: (8, 256, 256), 5: (4, 512, 512), 6: (2, 512, 512)}
# (block, mode, bm, bn, bk, kg, splits)
CONFIGS = [(3, 0, 64, 64, 64, 2, 1), (3, 0, 128, 128, 32, 2, 4), (5, 2, 128, 128, 32, 2, 1), (5, 0, 128, 64, 32, 1, 4),
           (6, 1, 64, 64, 64, 1, 8)]
WS = torch.empty(16 << 20, device=dev)
for (l, mode, bm, bn, bk, kg, sp) in CONFIGS:
    H, cin, cout = BLOCKS[l]
    x3 = Fn.split3(torch.randn(B, H, H, cin, device=dev))
    w3 = Fn.split3(torch.randn(cout, 3, 3, cin, device=dev) * 0.05)
    dz3 = Fn.split3(torch.randn(B * H * H, cout, device=dev))
    M, N, K = Fn.gemm_dims(mode, B, H, H, cin, cout)
    out = torch.empty(max(M * N, cout * 9 * cin), device=dev)
    for _ in range(5):
        C.conv_gemm_xp(mode, x3 if mode != 1 else None, w3 if mode != 2 else None, dz3 if mode != 0 else None, None,
                       out, WS, None, B, H, H, cin, cout, bm, bn, sp, bk, kg)
    torch.cuda.synchronize()
print("done")
