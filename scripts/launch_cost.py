"""Device-side cost of a dependent chain of tiny kernels on one stream (the floor every launch on the
VGG step's critical chain pays): N one-element kernels captured in a HIP graph and replayed, vs the
same N launched eagerly; plus the same with a second stream busy (side-stream work next to the chain).

    python scripts/launch_cost.py [--n 1000]
"""
import argparse
import json

import torch


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=1000)
    a = p.parse_args()
    x = torch.zeros(1, device="cuda")
    out = {}
    # eager
    for _ in range(50):
        x.add_(1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.n):
        x.add_(1)
    e1.record()
    e1.synchronize()
    out["eager_us_per_kernel"] = round(e0.elapsed_time(e1) * 1e3 / a.n, 3)
    # graph
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(a.n):
                x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    out["graph_us_per_kernel"] = round(e0.elapsed_time(e1) * 1e3 / a.n, 3)
    # a medium kernel chain: 1 MiB elementwise (bandwidth trivial) eager
    y = torch.zeros(1 << 18, device="cuda")
    for _ in range(50):
        y.add_(1)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.n):
        y.add_(1)
    e1.record()
    e1.synchronize()
    out["eager_1MiB_us_per_kernel"] = round(e0.elapsed_time(e1) * 1e3 / a.n, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
