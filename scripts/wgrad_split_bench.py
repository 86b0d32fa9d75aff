"""Weight-gradient GEMM dW = dY^T . col ([Co, M] x [M, K], bf16 in, fp32 out) at ResNet-50 B=256 shapes:
ops/cnn_nhwc._wgrad (row-chunk split as one batched GEMM + sum) vs one torch.mm(out_dtype=float32),
CUDA-event timed. One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc  # noqa: E402

dev = torch.device("cuda", 0)
B = 256
# (H*W rows per image, Co, K)
SHAPES = [(3136, 64, 256), (3136, 256, 64), (3136, 64, 64), (3136, 64, 576), (784, 128, 512), (784, 512, 128),
          (784, 128, 1152), (196, 256, 1024), (196, 1024, 256), (196, 256, 2304), (49, 512, 2048), (49, 2048, 512),
          (49, 512, 4608)]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / it


for hw, co, k in SHAPES:
    M = B * hw
    dy = torch.randn(M, co, device=dev).to(torch.bfloat16)
    col = torch.randn(M, k, device=dev).to(torch.bfloat16)
    a = timed(lambda: cnn_nhwc._wgrad(dy, col))
    b = timed(lambda: torch.mm(dy.t(), col, out_dtype=torch.float32))
    print(json.dumps({"M": M, "Co": co, "K": k, "splits": cnn_nhwc._wgrad_splits(M, co, k), "split_bmm_sum_us": round(a, 1),
                      "mm_fp32_us": round(b, 1)}), flush=True)
