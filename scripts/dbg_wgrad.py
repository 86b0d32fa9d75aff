import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from cs744_pytorch_distributed_tutorial_amd.ops import native
C = native.C()
dev = torch.device("cuda", 0)
P = 32 * 32
x = torch.zeros(1, 32, 32, 32, device=dev)
x[..., 0] = 1.0
dy = torch.arange(64, device=dev).float().view(1, 1, 1, 64).expand(1, 32, 32, 64).contiguous()
dw = C.conv_nhwc_bf16(2, dy.to(torch.bfloat16), x.to(torch.bfloat16), 1, 1, 1, 0, 0, 0)
print("rows (expect 0..63):", (dw[:, 0] / P).round().int().tolist())
# columns: dy = 1 for co == 0 only; x[p][c] = c
x2 = torch.arange(32, device=dev).float().view(1, 1, 1, 32).expand(1, 32, 32, 32).contiguous()
dy2 = torch.zeros(1, 32, 32, 64, device=dev); dy2[..., 0] = 1.0
dw2 = C.conv_nhwc_bf16(2, dy2.to(torch.bfloat16), x2.to(torch.bfloat16), 1, 1, 1, 0, 0, 0)
print("cols (expect 0..31):", (dw2[0] / P).round().int().tolist())
# pixel dependence: dy[p][co] = 1 for co==0, x[p][0] = p % 7
x3 = torch.zeros(1, 32, 32, 32, device=dev); x3[..., 0] = (torch.arange(P, device=dev) % 7).float().view(1, 32, 32)
dw3 = C.conv_nhwc_bf16(2, dy2.to(torch.bfloat16), x3.to(torch.bfloat16), 1, 1, 1, 0, 0, 0)
print("pix sum:", dw3[0, 0].item(), "expect", float((torch.arange(P) % 7).sum()))
# Co = 128: the 128-row tile
dy = torch.arange(128, device=dev).float().view(1, 1, 1, 128).expand(1, 32, 32, 128).contiguous()
dw = C.conv_nhwc_bf16(2, dy.to(torch.bfloat16), x.to(torch.bfloat16), 1, 1, 1, 0, 0, 0)
print("rows128 (expect 0..127):", (dw[:, 0] / P).round().int().tolist())
