"""Explicit gradient-synchronisation strategies (the subject of the tutorial).

Each strategy runs after ``loss.backward()`` and before ``optimizer.step()``:

==================  ========================================================  ======================================
name                reference                                                 behaviour
==================  ========================================================  ======================================
``gather_scatter``  part2a (`master/part2a/part2a.py:42-52`,                   per parameter: gather to rank 0, mean
                    `slave/part2a/part2a.py:43-45`)                           on rank 0, scatter the mean back
``p2p``             part2a_extra (`master/part2a/part2a_extra.py:41-58`,       per parameter star: rank 0 receives from
                    `slave/part2a/part2a_extra.py:41-45`)                     every rank, averages, sends back
``allreduce``       part2b (`master/part2b/part2b.py:43-45`)                  per parameter ``grad/N`` then
                                                                              ``all_reduce(SUM)``
``flat``            — (MI355X extension)                                      one coalesced ``all_reduce(AVG)``
==================  ========================================================  ======================================

DDP (part3) is `parallel.ddp.DistributedDataParallel` (hook-driven, overlapped).

The faithful modes keep the reference's *communication pattern* (one
collective per parameter tensor, rank-0 root, serialised p2p) so the tutorial's
lesson — DDP > all_reduce > star ≈ gather/scatter — is reproducible on RCCL.
Deviations, all documented: world size is not hard-coded to 4; the p2p star uses
``Work.wait()`` per message exactly like the reference but loops over the actual
world; ``coalesce=True`` variants batch each mode's messages into flat buffers.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

from .. import distributed as D


class GradSync:
    name = "none"

    def __init__(self, params: Sequence[torch.nn.Parameter], group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.rank = D.get_rank()
        self.world = D.get_world_size(group)

    def __call__(self) -> None:
        pass


class NoSync(GradSync):
    name = "none"


class GatherScatterSync(GradSync):
    """part2a: gather -> mean on root -> scatter, one pair per parameter."""

    name = "gather_scatter"

    def __init__(self, params, group=None, root: int = 0, coalesce: bool = False):
        super().__init__(params, group)
        self.root, self.coalesce = root, coalesce

    def _one(self, g: torch.Tensor) -> None:
        with _dense(g) as g:
            self._one_dense(g)

    def _one_dense(self, g: torch.Tensor) -> None:
        if self.rank == self.root:
            grad_list = [torch.zeros_like(g) for _ in range(self.world)]
            D.gather(g, grad_list, dst=self.root, group=self.group)
            mean = torch.stack(grad_list).sum(0).div_(self.world)
            D.scatter(g, [mean] * self.world, src=self.root, group=self.group)
        else:
            D.gather(g, dst=self.root, group=self.group)
            D.scatter(g, src=self.root, group=self.group)

    def __call__(self) -> None:
        if self.world == 1:
            return
        if self.coalesce:
            flat = torch.cat([p.grad.reshape(-1) for p in self.params])
            self._one(flat)
            _unflatten_into(flat, [p.grad for p in self.params])
        else:
            for p in self.params:
                self._one(p.grad)


class StarP2PSync(GradSync):
    """part2a_extra: rank 0 receives every rank's grad, averages, sends back."""

    name = "p2p"

    def __init__(self, params, group=None, root: int = 0, coalesce: bool = False, serialize: bool = True):
        super().__init__(params, group)
        self.root, self.coalesce, self.serialize = root, coalesce, serialize

    def _one(self, g: torch.Tensor) -> None:
        with _dense(g) as g:
            self._one_dense(g)

    def _one_dense(self, g: torch.Tensor) -> None:
        others = [r for r in range(self.world) if r != self.root]
        if self.rank == self.root:
            bufs = [torch.zeros_like(g) for _ in others]
            if self.serialize:  # reference: irecv(...).wait() one by one
                for r, b in zip(others, bufs):
                    D.irecv(b, src=r).wait()
            else:
                ops = [D.P2POp(torch.distributed.irecv, b, r) for r, b in zip(others, bufs)]
                for w in D.batch_isend_irecv(ops):
                    w.wait()
            for b in bufs:
                g.add_(b)
            g.div_(self.world)
            if self.serialize:
                for r in others:
                    D.isend(g, dst=r).wait()
            else:
                ops = [D.P2POp(torch.distributed.isend, g, r) for r in others]
                for w in D.batch_isend_irecv(ops):
                    w.wait()
        else:
            D.isend(g, dst=self.root).wait()
            D.irecv(g, src=self.root).wait()

    def __call__(self) -> None:
        if self.world == 1:
            return
        if self.coalesce:
            flat = torch.cat([p.grad.reshape(-1) for p in self.params])
            self._one(flat)
            _unflatten_into(flat, [p.grad for p in self.params])
        else:
            for p in self.params:
                self._one(p.grad)


class PerParamAllReduceSync(GradSync):
    """part2b: ``p.grad = p.grad / N`` then ``all_reduce(SUM)`` per parameter."""

    name = "allreduce"

    def __call__(self) -> None:
        if self.world == 1:
            return
        for p in self.params:
            if p.grad.is_contiguous():
                p.grad = p.grad / self.world
                D.all_reduce(p.grad, op=D.reduce_op.SUM, group=self.group, async_op=False)
            else:  # channels_last conv grads: collectives need a dense standard-layout tensor
                g = p.grad.contiguous().div_(self.world)
                D.all_reduce(g, op=D.reduce_op.SUM, group=self.group, async_op=False)
                p.grad.copy_(g)


class FlatAllReduceSync(GradSync):
    """One coalesced average all-reduce after backward (no overlap)."""

    name = "flat"

    def __call__(self) -> None:
        if self.world == 1:
            return
        grads = [p.grad for p in self.params]
        flat = torch.cat([g.reshape(-1) for g in grads])
        D.all_reduce(flat, op=D.ReduceOp.AVG, group=self.group)
        _unflatten_into(flat, grads)


class _dense:
    """Context: a contiguous alias of ``g`` (channels_last grads get a dense copy that is
    written back on exit), since gloo / RCCL collectives need standard-layout tensors."""

    def __init__(self, g: torch.Tensor):
        self.g = g
        self.c = g if g.is_contiguous() else g.contiguous()

    def __enter__(self) -> torch.Tensor:
        return self.c

    def __exit__(self, *exc) -> None:
        if self.c is not self.g:
            self.g.copy_(self.c)


def _unflatten_into(flat: torch.Tensor, tensors: List[torch.Tensor]) -> None:
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


SYNC_MODES = {
    "none": NoSync,
    "gather_scatter": GatherScatterSync,
    "p2p": StarP2PSync,
    "allreduce": PerParamAllReduceSync,
    "flat": FlatAllReduceSync,
}


def make_sync(mode: str, params, group=None, **kw) -> GradSync:
    if mode == "ddp":
        return NoSync(params, group)
    if mode not in SYNC_MODES:
        raise ValueError(f"unknown sync mode {mode!r}; choose from {sorted(SYNC_MODES) + ['ddp']}")
    return SYNC_MODES[mode](params, group, **kw)
