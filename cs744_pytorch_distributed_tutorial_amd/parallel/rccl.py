"""Python face of the native C++ RCCL communicator (``csrc/runtime/rccl_comm.cpp``).

The unique id is created by rank 0 and shared through the existing process group
(``broadcast_object_list`` rides the c10d store / gloo / RCCL, whichever backs
the default group), then every rank builds one ``ncclComm_t`` on its own GPU.
All collectives are enqueued on a dedicated high-priority comm stream after an
event wait on torch's current stream and never block the host; ``Handle.wait``
makes the current stream wait for the comm stream (no host sync).

Replaces the reference's gloo process group on the gradient data path
(`master/part2b/part2b.py:73-78`).
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import distributed as D
from ..ops import native
from .comm import Comm, Handle


class _RcclHandle(Handle):
    def __init__(self, comm):
        self.comm = comm

    def wait(self) -> None:
        self.comm.join()


class RcclComm(Comm):
    kind = "rccl"

    def __init__(self, native_comm):
        self.native = native_comm
        self.rank = native_comm.rank
        self.world_size = native_comm.world_size

    @classmethod
    def create(cls, rank: int, world: int, device: int, uid: Optional[bytes] = None, max_ctas: int = 0) -> "RcclComm":
        if uid is None:
            if world != 1:
                raise ValueError("RcclComm.create: a shared unique id is required for world > 1")
            uid = native.C().rccl_unique_id()
        return cls(native.C().RcclComm(uid, rank, world, device, True, int(max_ctas)))

    # construction in the three steps comm._agreed agrees on: local preparation, the collective
    # exchange of the unique id, then ncclCommInitRankConfig
    @staticmethod
    def prepare(group=None) -> Optional[bytes]:
        """Local only: load the extension, select the device; rank 0 creates the unique id."""
        C = native.C()
        torch.cuda.current_device()
        return C.rccl_unique_id() if D.get_rank(group) == 0 else None

    @staticmethod
    def share_uid(uid: Optional[bytes], group=None) -> bytes:
        obj = [uid]
        if D.get_world_size(group) > 1:
            torch.distributed.broadcast_object_list(obj, src=0, group=group)
        return obj[0]

    @classmethod
    def build(cls, uid: bytes, group=None, max_ctas: int = 0) -> "RcclComm":
        rank, world = D.get_rank(group), D.get_world_size(group)
        return cls(native.C().RcclComm(uid, rank, world, torch.cuda.current_device(), True, int(max_ctas)))

    @classmethod
    def from_process_group(cls, group=None, max_ctas: int = 0) -> "RcclComm":
        return cls.build(cls.share_uid(cls.prepare(group), group), group, max_ctas)

    # ---- Comm interface (all stream-ordered; handles join the comm stream back)
    def all_reduce_avg(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        self.native.all_reduce(buf, "avg")
        h = _RcclHandle(self.native)
        if not async_op:
            h.wait()
        return h

    def all_reduce_sum(self, buf: torch.Tensor, async_op: bool = True) -> Handle:
        self.native.all_reduce(buf, "sum")
        h = _RcclHandle(self.native)
        if not async_op:
            h.wait()
        return h

    def all_reduce(self, buf: torch.Tensor, op: str = "sum") -> None:
        self.native.all_reduce(buf, op)
        self.native.join()

    def broadcast(self, buf: torch.Tensor, src: int = 0) -> None:
        self.native.broadcast(buf, src)
        self.native.join()

    def all_gather_int64(self, values: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.world_size * values.numel(), dtype=values.dtype, device=values.device)
        self.native.all_gather(values.contiguous(), out)
        self.native.join()
        return out.view(self.world_size, -1)

    def gather_flat(self, buf: torch.Tensor, out: Optional[torch.Tensor], dst: int = 0) -> None:
        self.native.gather(buf, out, dst)
        self.native.join()

    def scatter_flat(self, buf: torch.Tensor, rows: Optional[torch.Tensor], src: int = 0) -> None:
        self.native.scatter(rows if self.rank == src else None, buf, src)
        self.native.join()

    def send(self, buf: torch.Tensor, dst: int) -> None:
        self.native.send(buf, dst)
        self.native.join()

    def recv(self, buf: torch.Tensor, src: int) -> None:
        self.native.recv(buf, src)
        self.native.join()

    def join(self) -> None:
        self.native.join()

    def check(self) -> None:
        err = self.native.async_error()
        if err:
            raise RuntimeError(f"RCCL async error: {err}")
