"""debug: WGRAD A staging of conv_nhwc_bf16 (mode 2)"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from cs744_pytorch_distributed_tutorial_amd.ops import native
C = native.C()
dev = torch.device("cuda", 0)
bf = torch.bfloat16
H, W, Co = 4, 8, 64
P = H * W
x = torch.zeros(1, H, W, 32, device=dev); x.view(P, 32)[0, 0] = 1.0
dy = torch.arange(Co, device=dev).float().view(1, 1, 1, Co).expand(1, H, W, Co).contiguous().to(bf)
print("dy[0,0,0,:16]", dy[0, 0, 0, :16].float().tolist(), dy.stride(), dy.is_contiguous())
dw = C.conv_nhwc_bf16(2, dy, x.to(bf), 1, 1, 1, 0, 0, 0)
torch.cuda.synchronize()
print("col0:", dw[:, 0].round().int().tolist()[:16])
