"""Collective bus-bandwidth sweep (nccl-tests conventions) over the framework's comms.

BASELINE.json names "all-reduce bus BW" as part of the headline metric; the reference
only ever measured it implicitly (its gloo all_reduce of the 35.21 MiB VGG-11 gradient,
`master/part2b/part2b.py:43-45`; BASELINE.md rows "all_reduce bus BW"). This sweeps
message sizes for one collective and prints one JSON line per size:

    algbw = bytes / time,   busbw = algbw * factor(op, N)
    factor: all_reduce 2(N-1)/N, all_gather / reduce_scatter (N-1)/N, broadcast 1

Backends: ``--comm rccl`` = the native C++ RcclComm (stream-ordered, ncclAvg/Sum on a
dedicated comm stream — the DDP data plane), ``--comm torch`` = torch.distributed
(ProcessGroupNCCL = RCCL on GPU tensors, gloo on CPU tensors). ``--device cpu`` runs
gloo (the reference's transport) so the same sweep reproduces the BASELINE.md rows.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m \\
        cs744_pytorch_distributed_tutorial_amd.bench.busbw --op all_reduce --comm rccl
Also the ``--vgg-buckets`` mode: the VGG-11 gradient (9,231,114 fp32) split into the
engine's DDP bucket plan, all-reduced back to back (what one training step sends).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List

import torch

from .. import distributed as D

FACTORS = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
}

def _sig(x: float) -> float:
    """4 significant digits (a fixed 3-decimal round turns a slow gloo 4 KiB op into 0)."""
    return float(f"{x:.4g}")


VGG11_GRAD_FLOATS = 9_231_114


def parse_size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def default_sizes(device: str) -> List[int]:
    hi = 256 << 20 if device == "cuda" else 64 << 20
    out, s = [], 4 << 10
    while s <= hi:
        out.append(s)
        s *= 4
    return out


class _Runner:
    """One collective on a fixed buffer; ``issue()`` enqueues, ``sync()`` completes."""

    def __init__(self, op: str, comm: str, nbytes: int, device: torch.device, world: int):
        self.op, self.world, self.device = op, world, device
        # nccl-tests convention: the size is the full vector (all_gather's output,
        # reduce_scatter's input), so per-rank shards are size / N
        n = max(1, nbytes // 4)
        shard = max(1, n // world)
        self.buf = torch.ones(n, dtype=torch.float32, device=device)
        self.out = None
        if op == "all_gather":
            self.buf = torch.ones(shard, dtype=torch.float32, device=device)
            self.out = torch.empty(shard * world, dtype=torch.float32, device=device)
        elif op == "reduce_scatter":
            self.buf = torch.ones(shard * world, dtype=torch.float32, device=device)
            self.out = torch.empty(shard, dtype=torch.float32, device=device)
        self.nbytes = (self.out.numel() if op == "all_gather" else self.buf.numel()) * 4
        self.native = None
        if comm == "rccl":
            if device.type != "cuda":
                raise ValueError("--comm rccl needs GPU tensors")
            from ..parallel.rccl import RcclComm
            self.native = RcclComm.from_process_group().native

    def issue(self):
        c = self.native
        if c is not None:
            if self.op == "all_reduce":
                c.all_reduce(self.buf, "sum")
            elif self.op == "broadcast":
                c.broadcast(self.buf, 0)
            elif self.op == "all_gather":
                c.all_gather(self.buf, self.out)
            else:
                c.reduce_scatter(self.buf, self.out, "sum")
            return
        if self.op == "all_reduce":
            D.all_reduce(self.buf, op=D.ReduceOp.SUM)
        elif self.op == "broadcast":
            D.broadcast(self.buf, src=0)
        elif self.op == "all_gather":
            D.all_gather_into_tensor(self.out, self.buf)
        else:
            D.reduce_scatter_tensor(self.out, self.buf, op=D.ReduceOp.SUM)

    def sync(self):
        if self.native is not None:
            self.native.join()
        if self.device.type == "cuda":
            torch.cuda.synchronize()


def time_op(run: _Runner, iters: int, warmup: int) -> float:
    """Seconds per collective: max over ranks of the mean over ``iters`` back-to-back calls."""
    for _ in range(warmup):
        run.issue()
    run.sync()
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        run.issue()
    run.sync()
    dt = (time.perf_counter() - t0) / iters
    return D.all_reduce_scalar(dt, op=D.ReduceOp.MAX) if D.get_world_size() > 1 else dt


def bucket_plan_sizes(bucket_mb: float) -> List[int]:
    """Byte sizes of the native engine's VGG-11 DDP buckets (layer-aligned, from the top)."""
    from ..runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    _, ranges = lay.plan_buckets(bucket_mb)
    return [n * 4 for _, n in ranges]


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--op", default="all_reduce", choices=sorted(FACTORS))
    p.add_argument("--comm", default="rccl", choices=["rccl", "torch"])
    p.add_argument("--device", default=None, choices=["cuda", "cpu"])
    p.add_argument("--sizes", default=None, help="comma list, e.g. 4K,1M,35.21M (default 4 KiB .. 256 MiB x4)")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--vgg-buckets", type=float, default=None, metavar="MB",
                   help="time one step's worth of VGG-11 DDP buckets (cap MB) instead of a size sweep")
    p.add_argument("--json-out", default=None)
    a = p.parse_args(argv)
    device_kind = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    if device_kind == "cpu":
        a.comm = "torch"
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1 or not D.is_initialized():
        D.init_process_group(backend="nccl" if device_kind == "cuda" else "gloo")
    rank, world = D.get_rank(), D.get_world_size()
    device = D.device() if device_kind == "cuda" else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    rows = []
    if a.vgg_buckets is not None:
        sizes = bucket_plan_sizes(a.vgg_buckets)
        runs = [_Runner("all_reduce", a.comm, s, device, world) for s in sizes]
        for r in runs:
            for _ in range(a.warmup):
                r.issue()
            r.sync()
        D.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            for r in runs:
                r.issue()
        for r in runs:
            r.sync()
        dt = (time.perf_counter() - t0) / a.iters
        dt = D.all_reduce_scalar(dt, op=D.ReduceOp.MAX) if world > 1 else dt
        tot = sum(sizes)
        alg = tot / dt / 1e9
        rows.append({"bench": "vgg11_ddp_buckets", "comm": a.comm, "device": device.type, "n": world,
                     "bucket_mb": a.vgg_buckets, "buckets": len(sizes), "bytes": tot, "time_us": round(dt * 1e6, 2),
                     "algbw_GBps": _sig(alg), "busbw_GBps": _sig(alg * FACTORS["all_reduce"](world))})
    else:
        sizes = [parse_size(s) for s in a.sizes.split(",")] if a.sizes else default_sizes(device.type)
        for s in sizes:
            run = _Runner(a.op, a.comm, s, device, world)
            dt = time_op(run, a.iters, a.warmup)
            nbytes = run.nbytes
            alg = nbytes / dt / 1e9
            rows.append({"bench": "busbw", "op": a.op, "comm": a.comm, "device": device.type, "n": world,
                         "bytes": nbytes, "time_us": round(dt * 1e6, 2), "algbw_GBps": _sig(alg),
                         "busbw_GBps": _sig(alg * FACTORS[a.op](world))})
            del run
    if rank == 0:
        for r in rows:
            line = json.dumps(r)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "a") as f:
                    f.write(line + "\n")
    if world > 1:
        D.barrier()
    D.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
