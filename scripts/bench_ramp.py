"""Warm-up profile of the bench step: after W warmup steps, time consecutive windows of K
steps (each bracketed by a device sync) and print ms/step per window, plus the host time
to enqueue each window. Shows how many steps the step time takes to settle (clocks, queues)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd  # noqa: F401,E402  (sets the HIP queue count first)
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--window", type=int, default=20)
    p.add_argument("--windows", type=int, default=15)
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    t = NativeTrainer(batch_size=64, device=dev, graph="auto")
    for _ in range(a.warmup):
        t.step()
    torch.cuda.synchronize()
    rows = []
    for w in range(a.windows):
        t0 = time.perf_counter()
        for _ in range(a.window):
            t.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append({"window": w, "ms_per_step": round((t2 - t0) * 1e3 / a.window, 4),
                     "host_enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.window, 4)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
