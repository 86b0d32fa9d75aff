"""Warm-up profile of the bench step: after W warmup steps, time consecutive windows of K
steps (each bracketed by a device sync) and print ms/step per window, plus the host time
to enqueue each window. Shows how many steps the step time takes to settle (clocks, queues)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()  # before HIP starts, as bench.py does
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--window", type=int, default=20)
    p.add_argument("--windows", type=int, default=15)
    p.add_argument("--extra-streams", type=int, default=0,
                   help="create and use this many extra HIP streams first (more streams than hardware "
                        "queues: do the side-stream links still make progress when queues are shared?)")
    p.add_argument("--extra-after", action="store_true", help="create the extra streams after the trainer")
    p.add_argument("--reserve-first", action="store_true", help="reserve the engine's side stream before anything")
    p.add_argument("--nccl-pg", action="store_true",
                   help="first bring up a one-rank NCCL (RCCL) process group and run a barrier and an all-reduce "
                        "through it, as a multi-GPU job does before building its trainer")
    a = p.parse_args()
    if a.reserve_first:
        from cs744_pytorch_distributed_tutorial_amd.ops import native
        torch.cuda.set_device(0)
        native.C().reserve_streams()
    if a.nccl_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        torch.cuda.set_device(0)
        torch.distributed.init_process_group("nccl", rank=0, world_size=1)
        torch.distributed.barrier(device_ids=[0])
        x = torch.ones(4, device="cuda")
        torch.distributed.all_reduce(x)
        torch.cuda.synchronize()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    def make_extra():
        ex = [torch.cuda.Stream() for _ in range(a.extra_streams)]
        for st in ex:  # a kernel on every stream, so each is bound to a hardware queue
            with torch.cuda.stream(st):
                scratch.add_(1.0)
        torch.cuda.synchronize()
        return ex

    scratch = torch.zeros(1024, device=dev)
    extra = [] if a.extra_after else make_extra()
    t = NativeTrainer(batch_size=64, device=dev, graph="auto")
    from bench import _dpm_current, _sysfs_card
    card = _sysfs_card(dev)
    print(json.dumps({"sysfs_card": card, "sclk_mhz_idle": _dpm_current(os.path.join(card, "pp_dpm_sclk")) if card else None}), flush=True)
    if a.extra_after:
        extra = make_extra()
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
        if extra:  # keep the extra streams busy between windows too
            for st in extra:
                with torch.cuda.stream(st):
                    scratch.add_(1.0)
        rows.append({"window": w, "ms_per_step": round((t2 - t0) * 1e3 / a.window, 4),
                     "host_enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.window, 4),
                     "sclk_mhz": _dpm_current(os.path.join(card, "pp_dpm_sclk")) if card else None})
        print(json.dumps(rows[-1]), flush=True)
    t.check_comm()  # raises if a side-stream link wait timed out
    print("links ok", flush=True)


if __name__ == "__main__":
    main()
