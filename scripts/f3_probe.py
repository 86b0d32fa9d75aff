"""Price the F3 conv math (scaled fp16 hi/lo, 3 MFMAs; conv_gemm.hip "F3") in the VGG-11 step.

One process per run (cross-process A/B: run the arms alternately, several times each):
  python scripts/f3_probe.py --arm base        # the shipped tile table (X6S split-bf16 GEMMs)
  python scripts/f3_probe.py --arm f3probe     # the same tiles on F3, every operand bound read as 1.0
                                               # (VggEngine::set_f3_probe: WRONG numbers, timing only)
  python scripts/f3_probe.py --arm f3          # the same tiles on F3 with the producers' bounds
Prints one JSON line: arm, ms_per_step over the timed window, the tile stages used.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cs744_pytorch_distributed_tutorial_amd as pkg  # noqa: E402

pkg.ensure_hw_queues()
import torch  # noqa: E402

X6S, F3 = 16, 64


def to_f3(tr) -> int:
    """Every X6S GEMM of blocks >= 1 onto the same tile with the F3 math; returns how many."""
    n = 0
    C = tr.engine
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    for l in range(1, tr.layout.L):
        for m in range(3):
            bm, bn, sp, bk, st = C.get_tile(l, m)
            if st & X6S:
                nst = (st & ~X6S) | F3
                if native.C().conv_stage_ok(nst, bm, bn, bk, False):
                    C.set_tile(l, m, bm, bn, sp, bk, nst)
                    n += 1
    return n


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--arm", default="base",
                   help="base (the shipped table) | x6s (the v2 X6S table) | f3probe | f3 (X6S tiles on F3) | "
                        "tuned (the tile table in --table, key --key)")
    p.add_argument("--table", default="gpurun_out/tiles_tuned.json")
    p.add_argument("--key", default="VGG11/B64/gfx950/tuned")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    args = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=64, device=dev)
    n = 0
    if args.arm == "x6s":  # the round-5 v2 table (X6S maths)
        args.arm, args.table, args.key = "tuned", os.path.join(ROOT, "cs744_pytorch_distributed_tutorial_amd", "runtime",
                                                               "tiles_gfx950.json"), "VGG11/B64/gfx950/v2"
    if args.arm == "tuned":
        with open(args.table) as f:
            ent = json.load(f)[args.key]
        for t in ent["tiles"]:
            tr.engine.set_tile(*t[:6], t[6] if len(t) > 6 else 0)
        n = sum(1 for t in ent["tiles"] if len(t) > 6 and t[6] & F3)
    elif args.arm != "base":
        n = to_f3(tr)
        if args.arm == "f3probe":
            tr.engine.set_f3_probe(True)
    import gc
    gc.collect()
    gc.disable()
    for _ in range(args.warmup):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.steps
    print(json.dumps({"arm": args.arm, "ms_per_step": round(ms, 4), "img_s": round(64e3 / ms, 1), "f3_gemms": n,
                      "steps": args.steps, "warmup": args.warmup, "loss": round(tr.last_loss(), 4)}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
