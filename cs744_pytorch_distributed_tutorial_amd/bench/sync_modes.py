"""Training throughput of every gradient-sync strategy of the tutorial, one JSON line each.

The tutorial's pedagogical result is the ordering of its four data-parallel variants
(DDP > per-tensor all-reduce > p2p star ~ gather/scatter). This runs the
same VGG-11 step under each ``--modes`` entry and reports whole-job images/s:

* ``gather_scatter`` — part2a (`master/part2a/part2a.py:42-52`): per-tensor gather to
  rank 0, mean, scatter;
* ``p2p``            — part2a_extra (`master/part2a/part2a_extra.py:41-58`): star from
  blocking send/recv;
* ``allreduce``      — part2b (`master/part2b/part2b.py:43-45`): per-tensor all-reduce;
* ``flat``           — one all-reduce of the whole flat gradient after backward;
* ``ddp``            — part3 (`master/part3/part3.py:116`): bucketed all-reduce(AVG)
  overlapped with backward.

GPU: the native engine (``runtime.engine.NativeTrainer``) with the native RCCL comm
(``--comm rccl``) or torch.distributed (``--comm torch``). CPU: the autograd trainer over
gloo, i.e. the reference's own transport, for the BASELINE.md reproduction.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \\
        cs744_pytorch_distributed_tutorial_amd.bench.sync_modes --steps 50
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

from .. import distributed as D

MODES = ("gather_scatter", "p2p", "allreduce", "flat", "ddp")


def make(mode: str, a, device, rank: int, world: int):
    if device.type == "cuda":
        from ..runtime.engine import NativeTrainer
        return NativeTrainer(model=a.model, batch_size=a.batch_size, device=device, rank=rank, world=world,
                             sync=mode, comm=a.comm, bucket_mb=a.bucket_mb)
    from ..runtime.torch_trainer import TorchTrainer
    return TorchTrainer(a.model, a.batch_size, device, rank, world, sync=mode, comm="torch", bucket_mb=a.bucket_mb,
                        fused_sgd=False)


def run_mode(mode: str, a, device, rank: int, world: int) -> dict:
    tr = make(mode, a, device, rank, world)
    sync = (lambda: torch.cuda.synchronize()) if device.type == "cuda" else (lambda: None)
    for _ in range(a.warmup):
        tr.step()
    sync()
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step()
    sync()
    D.barrier()
    dt = time.perf_counter() - t0
    dt = D.all_reduce_scalar(dt, op=D.ReduceOp.MAX) if world > 1 else dt
    loss = tr.last_loss()
    if hasattr(tr, "close"):
        tr.close()
    return {"bench": "sync_modes", "mode": mode, "n": world, "device": device.type, "model": a.model,
            "per_gpu_batch": a.batch_size, "steps": a.steps, "ms_per_step": round(1e3 * dt / a.steps, 4),
            "images_per_s": round(a.batch_size * world * a.steps / dt, 2), "final_loss": round(loss, 4),
            "comm": a.comm if device.type == "cuda" else "gloo", "bucket_mb": a.bucket_mb}


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--modes", default=",".join(MODES))
    p.add_argument("--model", default="VGG11")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--bucket-mb", type=float, default=4.0)
    p.add_argument("--comm", default="rccl", choices=["rccl", "torch"])
    p.add_argument("--device", default=None, choices=["cuda", "cpu"])
    p.add_argument("--json-out", default=None)
    a = p.parse_args(argv)
    kind = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    D.init_process_group(backend="nccl" if kind == "cuda" else "gloo")
    rank, world = D.get_rank(), D.get_world_size()
    device = D.device() if kind == "cuda" else torch.device("cpu")
    if kind == "cuda":
        torch.cuda.set_device(device)
    for mode in a.modes.split(","):
        if mode not in MODES:
            raise SystemExit(f"unknown mode {mode!r}; choose from {MODES}")
        row = run_mode(mode, a, device, rank, world)
        if rank == 0:
            line = json.dumps(row)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "a") as f:
                    f.write(line + "\n")
    D.barrier()
    D.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
