#!/usr/bin/env python3
"""Headline benchmark: VGG-11 training throughput on synthetic CIFAR-10-shaped data.

Metric (BASELINE.json): images/sec for the WHOLE node, VGG-11, 3x32x32 -> 10
classes, per-GPU batch 64 (the reference's part2/part3 per-rank batch,
`master/part2b/part2b.py:20`), SGD(0.1, 0.9, 1e-4), one process per GPU,
data-parallel gradient averaging (part3 = DDP semantics) over RCCL/xGMI.
Weak scaling: per-GPU batch fixed, global batch = 64 * N.

Contract: ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env). W untimed
warmup steps, then EXACTLY K timed steps bracketed by barrier + device sync on
both sides; the max over ranks is reported; rank 0 prints ONE JSON line.

Every timed step does the full work: batch gather + augmentation on device,
forward, loss, backward, gradient all-reduce (N > 1), SGD update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from cs744_pytorch_distributed_tutorial_amd import distributed as D  # noqa: E402

# best reference configuration (part3 DDP, N=4, local CPU repro) = 554 img/s.
BASELINE_IMG_S = 554.0


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch-size", type=int, default=64, help="per-GPU batch")
    p.add_argument("--model", type=str, default="VGG11")
    p.add_argument("--engine", type=str, default=os.environ.get("CS744_BENCH_ENGINE", "native"),
                   choices=["torch", "native"])
    p.add_argument("--sync", type=str, default="ddp",
                   choices=["ddp", "allreduce", "gather_scatter", "p2p", "flat"])
    p.add_argument("--comm", type=str, default="rccl", choices=["torch", "rccl"])
    p.add_argument("--bucket-mb", type=float, default=9.0)
    p.add_argument("--bucket-policy", type=str, default="layer", choices=["size", "layer", "single"])
    p.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--no-graph", action="store_true", help="native engine: disable hipGraph capture")
    p.add_argument("--graph", type=str, default="auto", choices=["auto", "full", "segments", "none"])
    p.add_argument("--json-out", type=str, default=None)
    return p.parse_args(argv)


class TorchTrainer:
    """Stock-PyTorch path (MIOpen/hipBLASLt kernels via autograd) — the comparison baseline."""

    def __init__(self, args, device, rank, world):
        from cs744_pytorch_distributed_tutorial_amd.models import VGG
        from cs744_pytorch_distributed_tutorial_amd.parallel import DistributedDataParallel, make_comm, make_sync
        from cs744_pytorch_distributed_tutorial_amd.utils import data as dm
        torch.manual_seed(5000)
        self.model = VGG(args.model).to(device)
        self.world = world
        if world > 1 and args.sync == "ddp":
            self.net = DistributedDataParallel(self.model, comm=make_comm(args.comm), bucket_cap_mb=args.bucket_mb,
                                               bucket_policy=args.bucket_policy)
            self.sync = make_sync("none", [])
        else:
            self.net = self.model
            self.sync = make_sync(args.sync if world > 1 else "none", self.model.parameters())
        self.opt = torch.optim.SGD(self.net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
        self.crit = torch.nn.CrossEntropyLoss()
        ds = dm.SyntheticCIFAR10(train=True, size=50_000, seed=0)
        sampler = dm.DistributedSampler(len(ds), world, rank, shuffle=True, seed=0)
        self.loader = dm.DeviceDataLoader(ds, args.batch_size, sampler=sampler, train=True, device=device,
                                          drop_last=True)
        self._it = iter(self.loader)
        self.loss = None

    def _batch(self):
        try:
            return next(self._it)
        except StopIteration:
            self.loader.set_epoch(self.loader.epoch + 1)
            self._it = iter(self.loader)
            return next(self._it)

    def step(self):
        x, y = self._batch()
        self.opt.zero_grad()
        loss = self.crit(self.net(x), y)
        loss.backward()
        self.sync()
        self.opt.step()
        self.loss = loss.detach()

    def last_loss(self) -> float:
        return float(self.loss.item())


def make_trainer(args, device, rank, world):
    if args.engine == "torch":
        return TorchTrainer(args, device, rank, world)
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    return NativeTrainer.from_bench_args(args, device, rank, world)


def main(argv=None) -> int:
    args = parse(argv)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:
        D.init_process_group(backend="nccl")
    rank, world = D.get_rank(), D.get_world_size()
    if world != args.gpus and rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    device = D.device() if world > 1 else torch.device("cuda", 0)
    torch.cuda.set_device(device)
    trainer = make_trainer(args, device, rank, world)

    for _ in range(args.warmup):
        trainer.step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = D.all_reduce_scalar(elapsed, op=D.ReduceOp.MAX) if world > 1 else elapsed
    loss = trainer.last_loss()
    imgs = args.batch_size * world * args.steps
    value = imgs / elapsed
    out = {
        "metric": "images/sec (whole node) VGG-11 CIFAR-shape",
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_IMG_S, 2),
        "dtype": "fp32" if args.dtype == "fp32" else "bf16",
        "data": "synthetic (CIFAR-10 shape 3x32x32 uint8, on-device augmentation), random-init weights",
        "config": {"model": "VGG-11", "global_batch": args.batch_size * world, "per_gpu_batch": args.batch_size,
                   "seq_len": None, "parallelism": f"dp{world}", "sync": args.sync if world > 1 else "none",
                   "engine": args.engine, "comm": args.comm, "bucket_mb": args.bucket_mb,
                   "bucket_policy": args.bucket_policy, "optimizer": "SGD(lr=0.1, momentum=0.9, wd=1e-4)",
                   "final_loss": round(loss, 4), "baseline_img_s": BASELINE_IMG_S},
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "a") as f:
                f.write(line + "\n")
    if world > 1:
        D.barrier()
        D.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
