"""Python faces of the two non-RCCL native communicators (``csrc/runtime/staged_comm.h``).

* ``StagedComm`` — the engine's C++ ``DeviceComm`` contract over a c10d gloo group with
  host staging. It lets the exact C++ data-parallel step (``VggEngine::step``: bucket
  forks, the BN-buffer broadcast behind bucket 0, the join before SGD) run with N ranks
  that share ONE MI355X — RCCL refuses two ranks on one device ("Duplicate GPU
  detected", measured on the 1-GPU box) — so the multi-rank path of the N-GPU benchmark
  is tested without an N-GPU node. Python-level collectives (construction broadcast,
  faithful sync modes) go through the torch.distributed facade on the same group.
* ``ProbeComm`` — world 1; every collective is a spin plus an exact scramble/unscramble
  on the comm stream, so a missing fork/join in the engine is a bitwise mismatch.

Reference: the gloo process group of every distributed script (`master/part3/part3.py:69-74`),
whose role on the gradient path these stand in for in tests.
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import distributed as D
from ..ops import native
from .comm import Comm, TorchComm


def _gloo_group(group=None):
    """The gloo group to stage through: ``group`` itself, or the facade's gloo side group
    when the default backend is RCCL."""
    if D.get_backend(group) == "gloo":
        return group if group is not None else torch.distributed.group.WORLD
    return D._group_for(torch.zeros(1), group)


class StagedComm(TorchComm):
    kind = "staged"

    def __init__(self, group=None, device: Optional[int] = None):
        g = _gloo_group(group)
        super().__init__(g)
        dev = torch.cuda.current_device() if device is None else device
        self.native = native.C().StagedComm(g.group_name, dev)

    def join(self) -> None:
        self.native.join()

    def check(self) -> None:
        err = self.native.async_error()
        if err:
            raise RuntimeError(f"staged communicator error: {err}")


class ProbeComm(Comm):
    """World-1 ordering probe (no Python-level collectives: world 1)."""
    kind = "probe"

    def __init__(self, device: Optional[int] = None, spin_us: float = 20.0, gbps: float = 0.0, world: int = 8,
                 ctas: int = 0):
        """gbps > 0: the xGMI model (no scramble): every all-reduce spins spin_us plus the ring time
        of a ``world``-GPU ring at ``gbps`` bus bandwidth, every broadcast spin_us + bytes / gbps;
        ctas > 0: the spin is that many busy workgroups (an RCCL collective's CU footprint)."""
        dev = torch.cuda.current_device() if device is None else device
        self.native = native.C().ProbeComm(dev, spin_us, gbps, world, ctas)
        self.rank, self.world_size = 0, 1

    def broadcast(self, buf: torch.Tensor, src: int = 0) -> None:
        pass

    def join(self) -> None:
        self.native.join()

    def check(self) -> None:
        pass
