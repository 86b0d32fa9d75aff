"""ResNet-50 convolutions (B=256, bf16, NHWC) that the implicit-GEMM kernel serves: forward +
backward time of ops/cnn_nhwc.conv_nhwc with the implicit path vs the im2col + hipBLASLt path
(CS_CONV_IMPLICIT=0 vs 2), per layer shape, CUDA-event timed over repeated calls. One JSON line per
shape; a weighted total over the convs of one ResNet-50 step at the end."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
# (H, Cin, Cout, k, stride, count in one ResNet-50 forward)
SHAPES = [(56, 64, 64, 3, 1, 3), (56, 128, 128, 3, 2, 1), (28, 128, 128, 3, 1, 3), (28, 256, 256, 3, 2, 1),
          (14, 256, 256, 3, 1, 5), (14, 512, 512, 3, 2, 1), (7, 512, 512, 3, 1, 2), (56, 256, 512, 1, 2, 1),
          (28, 512, 1024, 1, 2, 1), (14, 1024, 2048, 1, 2, 1)]


def timed(H, Ci, Co, k, st, mode):
    os.environ["CS_CONV_IMPLICIT"] = mode
    dev = torch.device("cuda", 0)
    conv = torch.nn.Conv2d(Ci, Co, k, st, k // 2, bias=False).to(dev)
    x = torch.randn(B, H, H, Ci, device=dev).to(torch.bfloat16).requires_grad_()
    Ho = (H + 2 * (k // 2) - k) // st + 1
    g = torch.randn(B, Ho, Ho, Co, device=dev).to(torch.bfloat16)

    def once():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = cnn_nhwc.conv_nhwc(x, conv)
        y.backward(g)

    for _ in range(2):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(ITERS):
        once()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / ITERS


tot = {"0": 0.0, "2": 0.0}
for (H, Ci, Co, k, st, n) in SHAPES:
    r = {m: timed(H, Ci, Co, k, st, m) for m in ("0", "2")}
    for m in r:
        tot[m] += n * r[m]
    flop = 3 * 2.0 * B * ((H + 2 * (k // 2) - k) // st + 1) ** 2 * Co * Ci * k * k
    print(json.dumps({"H": H, "Cin": Ci, "Cout": Co, "k": k, "stride": st, "per_net": n, "im2col_us": round(r["0"], 1),
                      "implicit_us": round(r["2"], 1), "implicit_tflops": round(flop / r["2"] / 1e6, 1)}), flush=True)
print(json.dumps({"B": B, "total_im2col_us": round(tot["0"], 1), "total_implicit_us": round(tot["2"], 1)}), flush=True)
