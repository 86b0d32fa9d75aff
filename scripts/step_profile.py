"""Per-step device-time profile of a short bench window (why a 20-step window reads slower per
step than a 100-step one). After W warmup steps and the same barrier + device sync bench.py uses,
a HIP event is recorded on the compute stream before every step of a K-step window (and after the
last): prints each step's interval, the window's host enqueue time, and the gap between the window
start (host clock) and the first step's device start.

    python scripts/step_profile.py [--warmup 5] [--steps 20] [--windows 3]
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
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--windows", type=int, default=3)
    p.add_argument("--pretrain", type=int, default=0,
                   help="> 0: train that many steps first, then restore the initial parameters / momentum / "
                        "buffers / cursor (a ramp that comes back is a property of the training state)")
    p.add_argument("--prewarm-ms", type=float, default=0.0,
                   help="> 0: that long of bf16 GEMMs before the warmup steps (is the ramp the clock?)")
    p.add_argument("--host-sleep-us", type=float, default=0.0,
                   help="> 0: busy-wait this long on the host after each timed step's enqueue (does the "
                        "host's lead over the GPU change the device step time?)")
    p.add_argument("--second-trainer", type=int, default=0,
                   help="> 0: first run a throw-away trainer for this many steps (is the ramp per process or per trainer?)")
    p.add_argument("--prewarm-copy-ms", type=float, default=0.0,
                   help="> 0: that long of 256 MiB device copies before the warmup steps (is it the memory clock?)")
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    if a.second_trainer > 0:
        t0_ = NativeTrainer(batch_size=64, device=torch.device("cuda", 0))
        for _ in range(a.second_trainer):
            t0_.step()
        torch.cuda.synchronize()
        t0_.close()
        del t0_
    tr = NativeTrainer(batch_size=64, device=torch.device("cuda", 0))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import _sysfs_card, _dpm_current
    card = _sysfs_card(torch.device("cuda", 0))
    sclk = lambda: _dpm_current(os.path.join(card, "pp_dpm_sclk")) if card else None  # noqa: E731
    if a.prewarm_ms > 0:
        x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < a.prewarm_ms / 1e3:
            for _ in range(8):
                torch.mm(x, x)
            torch.cuda.synchronize()
    if a.pretrain > 0:
        snap = [t.clone() for t in (tr.params, tr.mom, tr.bufs, tr.nbt)]
        cur = tr.engine.cursor().clone()
        mom_valid, gstep = tr._mom_valid, tr.global_step
        for _ in range(a.pretrain):
            tr.step()
        torch.cuda.synchronize()
        for dst, src in zip((tr.params, tr.mom, tr.bufs, tr.nbt), snap):
            dst.copy_(src)
        tr.engine.cursor().copy_(cur)
        tr._mom_valid, tr.global_step = mom_valid, gstep
        torch.cuda.synchronize()
    if a.prewarm_copy_ms > 0:
        src = torch.empty(64 << 20, device="cuda")
        dst = torch.empty_like(src)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < a.prewarm_copy_ms / 1e3:
            for _ in range(4):
                dst.copy_(src)
            torch.cuda.synchronize()
        del src, dst
    import gc
    gc.collect()
    gc.disable()
    for _ in range(a.warmup):
        tr.step()
    for w in range(a.windows):
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
        t0 = time.perf_counter()
        for i in range(a.steps):
            ev[i].record()
            tr.step()
            if a.host_sleep_us > 0:
                t1 = time.perf_counter()
                while time.perf_counter() - t1 < a.host_sleep_us / 1e6:
                    pass
        ev[-1].record()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        per = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.steps)]
        print(json.dumps({"window": w, "sclk_mhz_after": sclk(), "wall_ms": round(1e3 * t_all, 3), "enqueue_ms": round(1e3 * t_enq, 3),
                          "device_ms": round(ev[0].elapsed_time(ev[-1]), 3),
                          "per_step_ms": [round(x, 3) for x in per]}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
