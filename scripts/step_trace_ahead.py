"""A kernel-trace step timeline that the profiler's host cost cannot distort.

Under `rocprofv3 --kernel-trace` every dispatch costs the host several extra microseconds, so a
traced bench run is host-bound (~0.9 ms per traced step against ~0.63 ms unprofiled:
profiles/r6_f3_timeline.txt) and the gaps on the main queue are the host's, not the schedule's.
Here the main stream is first held by a device-side sleep long enough for the host to enqueue
every traced step; the steps then run back to back from a full queue, as in an unprofiled run.
Run under the profiler, then `python3 scripts/step_timeline.py <dir> --last K`:

    rocprofv3 --kernel-trace -d gpurun_out/ahead -o run -- python3 scripts/step_trace_ahead.py
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
    p.add_argument("--warmup", type=int, default=80, help="untimed steps first (past the start-up ramp)")
    p.add_argument("--steps", type=int, default=12, help="steps enqueued behind the sleep")
    p.add_argument("--hold-ms", type=float, default=60.0, help="device sleep ahead of them")
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(batch_size=64, device=torch.device("cuda", 0))
    import gc
    gc.collect()
    gc.disable()
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    sclk_hz = 2.4e9  # s_memtime-based sleep: a few percent either way does not matter here
    t0 = time.perf_counter()
    torch.cuda._sleep(int(a.hold_ms * 1e-3 * sclk_hz))
    for _ in range(a.steps):
        tr.step()
    host_ms = 1e3 * (time.perf_counter() - t0)
    torch.cuda.synchronize()
    wall_ms = 1e3 * (time.perf_counter() - t0)
    # the hold only hides the host if the host finished enqueueing before the device got going
    print(json.dumps({"steps": a.steps, "hold_ms": a.hold_ms, "host_enqueue_ms": round(host_ms, 2),
                      "wall_ms": round(wall_ms, 2), "host_ahead": host_ms < a.hold_ms,
                      "loss": round(tr.last_loss(), 4)}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
