"""Communicator backends used by the gradient-sync engines.

``Comm`` is the small interface the bucketed reducer needs — asynchronous
average-all-reduce of a contiguous buffer plus broadcast — with two
implementations:

* ``TorchComm`` — ``torch.distributed`` (ProcessGroupNCCL = RCCL on GPU
  tensors, gloo on CPU tensors). RCCL work is enqueued on the process group's
  internal stream after an event wait on the caller's current stream, so a call
  issued right after a layer's weight-gradient kernel overlaps the rest of the
  backward pass; ``wait()`` only makes the current stream wait (no host block).
* ``RcclComm`` (``parallel.rccl``) — the native C++ communicator: one
  ``ncclComm_t`` built from a TCPStore-shared unique id, a dedicated high-priority
  comm stream, HIP events between compute and comm streams, ``ncclAvg`` so the
  1/N costs no extra kernel. Stream-ordered and host-sync-free, so it can be
  captured into a hipGraph together with the compute kernels.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import distributed as D


class Handle:
    def wait(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class _TorchHandle(Handle):
    def __init__(self, work):
        self.work = work

    def wait(self) -> None:
        if self.work is not None:
            self.work.wait()


class Comm:
    rank: int = 0
    world_size: int = 1

    def all_reduce_avg(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        raise NotImplementedError

    def all_reduce_sum(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        raise NotImplementedError

    def broadcast(self, buf: torch.Tensor, src: int = 0) -> None:
        raise NotImplementedError

    def all_gather_int64(self, values: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    # flat-buffer primitives used by ``parallel.flat_sync`` (blocking w.r.t. the caller's stream)
    def all_reduce(self, buf: torch.Tensor, op: str = "sum") -> None:
        raise NotImplementedError

    def gather_flat(self, buf: torch.Tensor, out: Optional[torch.Tensor], dst: int = 0) -> None:
        """``out`` (on ``dst`` only) receives ``world * buf.numel()`` elements, rank-major."""
        raise NotImplementedError

    def scatter_flat(self, buf: torch.Tensor, rows: Optional[torch.Tensor], src: int = 0) -> None:
        """``buf`` receives row ``rank`` of ``rows`` (``world * buf.numel()`` elements, on ``src``
        only)."""
        raise NotImplementedError

    def send(self, buf: torch.Tensor, dst: int) -> None:
        raise NotImplementedError

    def recv(self, buf: torch.Tensor, src: int) -> None:
        raise NotImplementedError

    def join(self) -> None:
        """Make the caller's current stream wait for all communication issued so far."""


_OPS = {"sum": D.ReduceOp.SUM, "avg": D.ReduceOp.AVG, "max": D.ReduceOp.MAX, "min": D.ReduceOp.MIN}


class TorchComm(Comm):
    kind = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = D.get_rank(group)
        self.world_size = D.get_world_size(group)

    def all_reduce_avg(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        if self.world_size == 1:
            return _TorchHandle(None)
        return _TorchHandle(D.all_reduce(buf, op=D.ReduceOp.AVG, group=self.group, async_op=async_op))

    def all_reduce_sum(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        if self.world_size == 1:
            return _TorchHandle(None)
        return _TorchHandle(D.all_reduce(buf, op=D.ReduceOp.SUM, group=self.group, async_op=async_op))

    def broadcast(self, buf: torch.Tensor, src: int = 0) -> None:
        if self.world_size > 1:
            D.broadcast(buf, src=src, group=self.group)

    def all_gather_int64(self, values: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return values.reshape(1, -1)
        out = [torch.zeros_like(values) for _ in range(self.world_size)]
        D.all_gather(out, values, group=self.group)
        return torch.stack(out)

    def all_reduce(self, buf: torch.Tensor, op: str = "sum") -> None:
        if self.world_size > 1:
            D.all_reduce(buf, op=_OPS[op], group=self.group)  # the facade maps AVG to SUM+scale on gloo

    def gather_flat(self, buf: torch.Tensor, out: Optional[torch.Tensor], dst: int = 0) -> None:
        if self.world_size == 1:
            if out is not None:
                out.copy_(buf.reshape(-1))
            return
        lst = list(out.view(self.world_size, -1).unbind(0)) if self.rank == dst else None
        D.gather(buf, lst, dst=dst, group=self.group)

    def scatter_flat(self, buf: torch.Tensor, rows: Optional[torch.Tensor], src: int = 0) -> None:
        if self.world_size == 1:
            if rows is not None:
                buf.copy_(rows.reshape(-1)[:buf.numel()])
            return
        lst = list(rows.view(self.world_size, -1).unbind(0)) if self.rank == src else None
        D.scatter(buf, lst, src=src, group=self.group)

    def send(self, buf: torch.Tensor, dst: int) -> None:
        D.isend(buf, dst, group=self.group).wait()

    def recv(self, buf: torch.Tensor, src: int) -> None:
        D.irecv(buf, src, group=self.group).wait()


def _all_ok(ok: bool, group) -> bool:
    """One MIN all-reduce of a per-rank success flag over ``group`` (its backend's device)."""
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item()) == 1


def _agreed(build, group, what: str, prepare=None, share=None, fallback_comm=None) -> Comm:
    """Build a native communicator on every rank, or on none, in two agreed phases (a rank that
    cannot join must not leave its peers waiting inside a collective):

    1. ``prepare()`` — purely local (load the extension, create the RCCL unique id on rank 0, set
       the device); every rank reports success in one MIN all-reduce, and only if ALL succeeded
    2. ``share(ctx)`` — the collective exchange (the unique id's broadcast), then ``build(shared)``
       (``ncclCommInitRankConfig``), and a second MIN all-reduce on the outcome.
    Any failure in either phase takes every rank to ``fallback_comm()`` (default: the
    torch.distributed communicator).
    ``prepare``/``share`` default to no-ops, so ``build()`` alone gets the one-phase agreement."""
    import sys

    import torch.distributed as dist

    def fallback(err):
        comm = fallback_comm() if fallback_comm is not None else TorchComm(group)
        print(f"[comm] native {what} communicator unavailable on some rank ({err!r} here); "
              f"every rank falls back to {comm.kind}", file=sys.stderr, flush=True)
        return comm

    ctx, err = None, None
    try:
        ctx = prepare() if prepare is not None else None
    except Exception as e:  # noqa: BLE001 - reported, then agreed on below
        err = e
    if not dist.is_initialized():
        if err is not None:
            raise err
        shared = share(ctx) if share is not None else ctx
        return build(shared) if prepare is not None else build()
    if prepare is not None and not _all_ok(err is None, group):
        return fallback(err)
    comm = None
    try:
        if prepare is not None:
            shared = share(ctx) if share is not None else ctx
            comm = build(shared)
        else:
            comm = build()
    except Exception as e:  # noqa: BLE001
        err = e
    if _all_ok(err is None, group):
        return comm
    if comm is not None and hasattr(comm, "close"):
        comm.close()
    return fallback(err)


def comm_ctas() -> int:
    """RCCL compute budget (ncclConfig_t maxCTAs) for the native communicator: CS_COMM_CTAS, default
    16 — the bucketed all-reduces that overlap the backward then take at most 16 of the 256 CUs
    from the conv GEMMs; 0 leaves the choice to RCCL."""
    import os
    return int(os.environ.get("CS_COMM_CTAS", "16"))


def make_comm(kind: Optional[str] = None, group=None, max_ctas: Optional[int] = None) -> Comm:
    """``kind``: ``"torch"`` (default), ``"rccl"`` (native C++ RCCL communicator, one GPU per
    rank) or ``"staged"`` (native C++ communicator over a gloo group with host staging: the
    engine's C++ step with several ranks on one GPU, ``parallel.staged``)."""
    kind = kind or "torch"
    if kind == "torch":
        return TorchComm(group)
    if kind == "rccl":
        from .rccl import RcclComm

        def fallback_comm():
            # over a gloo control plane (bench.py's default at --comm rccl) the device buffers travel
            # through the staged communicator: the same C++ step, collectives host-staged over gloo
            import torch.distributed as dist
            if dist.is_initialized() and dist.get_backend(group) == "gloo" and torch.cuda.is_available():
                from .staged import StagedComm
                return StagedComm(group)
            return TorchComm(group)
        ctas = comm_ctas() if max_ctas is None else max_ctas
        return _agreed(lambda uid: RcclComm.build(uid, group, ctas), group, "rccl",
                       prepare=lambda: RcclComm.prepare(group), share=lambda uid: RcclComm.share_uid(uid, group),
                       fallback_comm=fallback_comm)
    if kind == "staged":
        from .staged import StagedComm
        return StagedComm(group)
    raise ValueError(f"unknown comm kind {kind!r}")
