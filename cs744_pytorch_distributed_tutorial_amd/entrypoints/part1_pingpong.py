"""part1 send/recv ping-pong (BASELINE.json config 1).

The reference's part1 has no communication at all; its send/recv usage lives
in part2a_extra (`master/part2a/part2a_extra.py:45-58`). This plumbing entrypoint
exercises exactly that surface — ``send``/``recv`` and ``isend``/``irecv`` +
``wait()`` between rank 0 and rank 1 — and reports round-trip latency and
bandwidth per message size. CPU/gloo by default (runs without a GPU);
``--device cuda`` uses RCCL over xGMI.

Correctness is checked on every round trip: rank 1 adds 1 to what it received
and sends it back; rank 0 verifies the values exactly.

    python -m cs744_pytorch_distributed_tutorial_amd.entrypoints.part1_pingpong \
        --master-ip 127.0.0.1 --num-nodes 2 --rank R
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

from .. import distributed as D
from ..config import add_reference_flags


def pingpong(sizes_bytes, iters: int = 20, warmup: int = 3, device: str = "cpu", use_async: bool = True) -> list:
    rank = D.get_rank()
    dev = torch.device(device) if device == "cpu" else D.device()
    rows = []
    for nbytes in sizes_bytes:
        n = max(1, nbytes // 4)
        buf = torch.zeros(n, dtype=torch.float32, device=dev)
        times = []
        for it in range(warmup + iters):
            if rank == 0:
                buf.copy_(torch.arange(n, dtype=torch.float32, device=dev) + it)
                t0 = time.perf_counter()
                if use_async:
                    D.isend(buf, dst=1).wait()
                    D.irecv(buf, src=1).wait()
                else:
                    D.send(buf, dst=1)
                    D.recv(buf, src=1)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                expect = torch.arange(n, dtype=torch.float32, device=dev) + it + 1
                if not torch.equal(buf, expect):
                    raise RuntimeError(f"ping-pong payload mismatch at size {nbytes}")
                if it >= warmup:
                    times.append(dt)
            elif rank == 1:
                if use_async:
                    D.irecv(buf, src=0).wait()
                    buf.add_(1)
                    D.isend(buf, dst=0).wait()
                else:
                    D.recv(buf, src=0)
                    buf.add_(1)
                    D.send(buf, dst=0)
        if rank == 0:
            times.sort()
            med = times[len(times) // 2]
            rows.append({"bytes": n * 4, "rtt_us": med * 1e6, "one_way_GBps": (n * 4) / (med / 2) / 1e9})
    return rows


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="send/recv ping-pong")
    add_reference_flags(p)
    p.add_argument("--port", type=int, default=29501)
    p.add_argument("--device", type=str, default="cpu", choices=["cpu", "cuda"])
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--sizes", type=str, default="8,1024,65536,1048576,9437184")
    p.add_argument("--blocking", action="store_true", help="use send/recv instead of isend/irecv+wait")
    a = p.parse_args(argv)
    backend = "gloo" if a.device == "cpu" else "nccl"
    D.init_process_group(backend=backend, rank=a.rank, world_size=a.num_nodes or 2, master_addr=a.master_ip,
                         master_port=a.port)
    if D.get_world_size() < 2:
        raise SystemExit("ping-pong needs world_size >= 2")
    rows = pingpong([int(s) for s in a.sizes.split(",")], iters=a.iters, device=a.device,
                    use_async=not a.blocking)
    if D.get_rank() == 0:
        for r in rows:
            print(json.dumps({"metric": "pingpong", "backend": backend, **r}))
    D.barrier()
    D.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
