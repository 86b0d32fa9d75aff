"""Autotune the VGG conv tile table on this GPU (every GEMM timed alone over every kernel variant
the engine has: tile, K-step, split-K, staging, maths incl. F3) and write it in the shipped-table
format (runtime/tiles_gfx950.json entries): python3 scripts/tune_tiles.py --out gpurun_out/tiles_tuned.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--key", default="VGG11/B64/gfx950/tuned")
    p.add_argument("--out", default="gpurun_out/tiles_tuned.json")
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr = NativeTrainer(batch_size=a.batch, device=dev, autotune=False)
    for _ in range(3):  # realistic operands (the F3 bounds need the producers to have run)
        tr.step()
    torch.cuda.synchronize()
    us = list(tr.engine.autotune(a.batch, a.iters))
    tiles = [[l, m] + list(tr.engine.get_tile(l, m)) for l in range(tr.layout.L) for m in range(3)
             if not (l == 0 and m == 1)]
    db = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            db = json.load(f)
    db[a.key] = {"tiles": tiles, "us": us, "tuner": "scripts/tune_tiles.py (VggEngine::autotune, each GEMM alone)"}
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1)
    for t in tr.tile_table():
        print(json.dumps(t))
    tr.close()


if __name__ == "__main__":
    main()
