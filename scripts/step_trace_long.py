"""Per-step device intervals over a long run with device syncs at chosen steps: does the step-time
ramp restart after every host sync (a property of the window bracket), or only at process start?

    python scripts/step_trace_long.py [--steps 240] [--sync-at 80,160] [--graph none]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=240)
    p.add_argument("--sync-at", default="80,160")
    p.add_argument("--sleep-ms", type=float, default=0.0, help="host sleep after each sync (GPU idle)")
    p.add_argument("--graph", default="none")
    a = p.parse_args()
    syncs = {int(x) for x in a.sync_at.split(",") if x}
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(batch_size=64, device=torch.device("cuda", 0), graph=a.graph)
    import gc
    gc.collect()
    gc.disable()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    torch.cuda.synchronize()
    for i in range(a.steps):
        if i in syncs:
            torch.cuda.synchronize()
            if a.sleep_ms > 0:
                time.sleep(a.sleep_ms / 1e3)
        ev[i].record()
        tr.step()
    ev[-1].record()
    torch.cuda.synchronize()
    per = [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(a.steps)]
    for i0 in range(0, a.steps, 20):
        blk = per[i0:i0 + 20]
        print(json.dumps({"steps": f"{i0}-{i0 + len(blk) - 1}", "mean_ms": round(sum(blk) / len(blk), 4),
                          "first3": blk[:3], "last3": blk[-3:]}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
