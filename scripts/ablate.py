"""In-process ablation / A-B of the native VGG step (one process, one trainer, variants interleaved
round by round — cdna_hip_programming.md §5.4 rule 24: cross-process variance looks like a kernel
property). A variant is an engine debug-skip mask (VggEngine::set_debug_skip: the upper bound of
what fusing away a launch class could save — WRONG numbers while set) and/or the serial backward.

    python scripts/ablate.py --variants "base:0" "no_fwd_apply:4" "no_fwd_fin:8" "serial:0:serial" \
        --rounds 5 --steps 50
Prints one JSON line per variant: median / min ms per step over the rounds."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cs744_pytorch_distributed_tutorial_amd as pkg  # noqa: E402

pkg.ensure_hw_queues()
import torch  # noqa: E402


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--variants", nargs="+", default=["base:0"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--model", default="VGG11")
    args = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(model=args.model, batch_size=args.batch_size, device=torch.device("cuda", 0), graph="none")
    base_overlap = tr.overlap_wgrad
    variants = []
    for v in args.variants:
        f = v.split(":")
        variants.append((f[0], int(f[1]) if len(f) > 1 and f[1] else 0, len(f) > 2 and f[2] == "serial"))
    import gc
    gc.collect()
    gc.disable()
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    times = {name: [] for name, _, _ in variants}
    for _ in range(args.rounds):
        for name, mask, serial in variants:
            tr.engine.set_debug_skip(mask)
            tr.engine.set_overlap(base_overlap and not serial)
            for _ in range(args.warmup):
                tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step()
            torch.cuda.synchronize()
            times[name].append(1e3 * (time.perf_counter() - t0) / args.steps)
    tr.engine.set_debug_skip(0)
    tr.engine.set_overlap(base_overlap)
    base = statistics.median(times[variants[0][0]])
    for name, mask, serial in variants:
        med = statistics.median(times[name])
        print(json.dumps({"variant": name, "mask": mask, "serial": serial, "ms_median": round(med, 4),
                          "ms_min": round(min(times[name]), 4), "img_s_median": round(args.batch_size * 1e3 / med, 1),
                          "delta_vs_first_pct": round(100.0 * (med - base) / base, 2),
                          "ms_all": [round(t, 4) for t in times[name]]}), flush=True)
    tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
