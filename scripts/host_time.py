"""Host enqueue time vs device time of the native VGG-11 step (B=64): is the eager C++ step
bound by the host's kernel launches? Prints per-step host time of trainer.step() (no sync) and
the device time per step over the same window, for the graph modes given on the command line."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as pkg

pkg.ensure_hw_queues()
import torch  # noqa: E402

from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer  # noqa: E402


def run(graph: str, steps: int = 60) -> None:
    dev = torch.device("cuda", 0)
    tr = NativeTrainer(batch_size=64, device=dev, train_size=50000, test_size=64, autotune=True, graph=graph)
    for _ in range(10):
        tr.step()
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(steps):
        h = time.perf_counter()
        tr.step()
        host.append(time.perf_counter() - h)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host.sort()
    print(f"graph={graph} overlap={tr.overlap_wgrad}: host enqueue per step median {1e3 * host[len(host) // 2]:.3f} ms "
          f"(p10 {1e3 * host[len(host) // 10]:.3f}), enqueue loop {1e3 * (t1 - t0) / steps:.3f} ms/step, "
          f"device {1e3 * (t2 - t0) / steps:.3f} ms/step (drain {1e3 * (t2 - t1):.2f} ms)", flush=True)
    del tr


for g in (sys.argv[1:] or ["none"]):
    run(g)
