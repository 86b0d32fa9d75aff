"""ResNet-50 stem (3 -> 64, 7x7/2, B x 224 x 224 image padded to 4 channels, bf16): forward and
forward + weight-gradient time of ops/cnn_nhwc.conv_nhwc, C4 implicit kernel (CS_CONV_IMPLICIT=1) vs
im2col + hipBLASLt (=0), CUDA-event timed. One JSON line per mode."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.ops import cnn_nhwc  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda", 0)
conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(dev)
x = cnn_nhwc.to_nhwc(torch.randn(B, 3, 224, 224, device=dev), torch.bfloat16, pad_c=1)
g = torch.randn(B, 112, 112, 64, device=dev).to(torch.bfloat16)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(ITERS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / ITERS


for mode in ("0", "1"):
    os.environ["CS_CONV_IMPLICIT"] = mode

    def fwd():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            cnn_nhwc.conv_nhwc(x, conv)

    def both():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = cnn_nhwc.conv_nhwc(x, conv)
        y.backward(g)

    print(json.dumps({"stem_impl": "implicit_c4" if mode == "1" else "im2col", "B": B,
                      "fwd_us": round(timed(fwd), 1), "fwd_wgrad_us": round(timed(both), 1)}), flush=True)
