"""BatchNorm backward kernels of the VGG-11 step timed alone (run under rocprofv3 --kernel-trace --stats):
is the apply pass slow by itself, or only next to the side stream's GEMMs? Shapes: B = 64, the
non-pool blocks 2, 4, 6 and the pooled blocks 1, 3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from cs744_pytorch_distributed_tutorial_amd.ops import functional as Fn
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for (H, C, pool) in ((8, 256, False), (4, 512, False), (2, 512, False), (16, 128, True), (8, 256, True)):
        B = 64
        M = B * H * H
        y = torch.randn(M, C, device=dev)
        Ho = H // 2 if pool else H
        G = torch.randn(B * Ho * Ho, C, device=dev)
        gamma = torch.rand(C, device=dev) + 0.5
        st = Fn.BNState(C, dev)
        st.scale.copy_(torch.rand(C, device=dev))
        st.shift.copy_(torch.randn(C, device=dev) * 0.1)
        st.mean.copy_(torch.randn(C, device=dev) * 0.1)
        st.invstd.copy_(torch.rand(C, device=dev) + 0.5)
        for _ in range(20):
            Fn.bn_relu_pool_bwd(y, G, st, gamma, B, H, H, pool=pool)
        torch.cuda.synchronize()
        print(f"H={H} C={C} pool={pool} elements={M * C}", flush=True)


if __name__ == "__main__":
    main()
