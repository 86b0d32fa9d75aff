"""DistributedDataParallel equivalent (reference part3, `master/part3/part3.py:116`;
semantics of torch's C++ ``Reducer``).

What it keeps from DDP:

* construction-time sync: parameter shapes are verified across ranks (one
  all-gather of a shape digest) and parameters + buffers are broadcast from
  rank 0 in one flattened message (N20);
* ``broadcast_buffers=True``: BN running stats / ``num_batches_tracked`` are
  broadcast from rank 0 before every training forward, and once before the
  first eval forward (N21, C-6b, C-7);
* bucketed, averaged all-reduce of gradients overlapped with backward (N19):
  gradients live in ONE flat buffer laid out in bucket order and every
  ``param.grad`` is a view into it (``gradient_as_bucket_view``), a
  post-accumulate-grad hook counts readiness, a full bucket is all-reduced
  asynchronously while autograd keeps computing earlier layers, and an
  end-of-backward callback waits for the last bucket. Buckets launch strictly in
  index order on every rank (RCCL needs identical collective order).
* ``state_dict`` keys carry the ``module.`` prefix, as with torch's DDP.

MI355X-native differences: bucket policy ``"layer"`` (xGMI-sized layer-aligned
buckets, `parallel.buckets`), ``ReduceOp.AVG`` (``ncclAvg``) instead of a separate
divide, and a pluggable communicator (``TorchComm`` or the native ``RcclComm``).

``grad_comm_dtype=torch.bfloat16`` (the default for the decoder-LM configs, runtime/torch_trainer.py):
each ready bucket's fp32 gradients are cast to bf16 (round to nearest even,
``csrc/kernels/flat_ops.hip`` cast_grad) on the compute stream, the all-reduce(AVG) runs on the
bf16 copy, and the average is widened back into the fp32 gradient view before the optimizer
reads it — half the bytes on the wire (Llama-3-8B pure DP: 16 GB instead of 32 GB of gradients
per step).
"""
from __future__ import annotations

import hashlib
from typing import List, Optional

import torch
import torch.nn as nn

from .buckets import Bucket, build_buckets
from .comm import Comm, make_comm


def _cast(src: torch.Tensor, dst: torch.Tensor) -> None:
    """fp32 <-> bf16 copy of one gradient bucket: the gfx950 cast kernel on the GPU (fails
    loudly if the extension is missing there), torch's copy_ (same rounding) on the CPU."""
    if src.is_cuda:
        from ..ops import native
        native.C().cast_grad(src, dst)
    else:
        dst.copy_(src)


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, comm: Optional[Comm] = None, bucket_cap_mb: float = 25.0,
                 first_bucket_cap_mb: float = 1.0, bucket_policy: str = "size",
                 broadcast_buffers: bool = True, sync_on_init: bool = True,
                 grad_comm_dtype: Optional[torch.dtype] = None):
        super().__init__()
        self.module = module
        self.comm = comm if comm is not None else make_comm("torch")
        self.broadcast_buffers = broadcast_buffers
        named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        self._names = [n for n, _ in named]
        self._params: List[nn.Parameter] = [p for _, p in named]
        if sync_on_init and self.comm.world_size > 1:
            self._verify_shapes()
            self._sync_module_states()
        self.buckets: List[Bucket] = build_buckets(self._params, policy=bucket_policy, cap_mb=bucket_cap_mb,
                                                   first_cap_mb=first_bucket_cap_mb, names=self._names)
        p0 = self._params[0]
        total = sum(b.numel for b in self.buckets)
        self.flat_grad = torch.zeros(total, dtype=p0.dtype, device=p0.device)
        # bf16 transport: the wire copy of every bucket (None: all-reduce the gradients in place)
        self.grad_comm_dtype = grad_comm_dtype if grad_comm_dtype not in (None, p0.dtype) else None
        if self.grad_comm_dtype is not None and (p0.dtype != torch.float32 or self.grad_comm_dtype != torch.bfloat16):
            raise ValueError("grad_comm_dtype: only bfloat16 transport of float32 gradients")
        self.flat_comm = torch.empty(total, dtype=self.grad_comm_dtype, device=p0.device) \
            if self.grad_comm_dtype is not None else None
        self._casts: List = []
        self._views: List[Optional[torch.Tensor]] = [None] * len(self._params)
        self._bucket_of = [0] * len(self._params)
        for b in self.buckets:
            for i, off in zip(b.param_indices, b.param_offsets):
                p = self._params[i]
                seg = self.flat_grad[off:off + p.numel()]
                # keep the parameter's own dense layout (channels_last conv weights), so the
                # gradient, the parameter and the fused optimizer's state all share strides
                self._views[i] = seg.as_strided(p.shape, p.stride()) if p.dim() == 4 and \
                    p.is_contiguous(memory_format=torch.channels_last) else seg.view_as(p)
                self._bucket_of[i] = b.index
        self._attach_grad_views(zero=True)
        self._pending = [0] * len(self.buckets)
        self._launched: List[bool] = [False] * len(self.buckets)
        self._ready: List[bool] = [False] * len(self.buckets)
        self._handles: List = []
        self._callback_queued = False
        self._buffers_synced_for_eval = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(self._params)]
        self._reset_counts()

    # ------------------------------------------------------------------ init sync
    def _verify_shapes(self) -> None:
        desc = ";".join(f"{n}:{tuple(p.shape)}:{p.dtype}" for n, p in zip(self._names, self._params))
        digest = int(hashlib.sha1(desc.encode()).hexdigest()[:15], 16)
        dev = self._params[0].device
        t = torch.tensor([digest, len(self._params)], dtype=torch.int64, device=dev)
        allv = self.comm.all_gather_int64(t)
        if not bool((allv == allv[0]).all()):
            raise RuntimeError(f"DDP: parameter shapes differ across ranks: {allv.tolist()}")

    def _state_tensors(self) -> List[torch.Tensor]:
        return [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]

    def _sync_module_states(self) -> None:
        """Broadcast params + buffers from rank 0, coalesced per dtype."""
        tensors = self._state_tensors()
        by_dtype = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            self.comm.broadcast(flat, src=0)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n

    def _sync_buffers(self) -> None:
        bufs = list(self.module.buffers())
        if not bufs or self.comm.world_size == 1:
            return
        by_dtype = {}
        for t in bufs:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            self.comm.broadcast(flat, src=0)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n

    # ------------------------------------------------------------------ grads
    def _attach_grad_views(self, zero: bool) -> None:
        need = any(p.grad is None or p.grad.data_ptr() != v.data_ptr() for p, v in zip(self._params, self._views))
        if need and zero:
            self.flat_grad.zero_()
        for p, v in zip(self._params, self._views):
            if p.grad is None:
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v

    def _reset_counts(self) -> None:
        for b in self.buckets:
            self._pending[b.index] = len(b.param_indices)
        self._launched = [False] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._handles = []
        self._callback_queued = False

    def _make_hook(self, i: int):
        def hook(p: torch.Tensor) -> None:
            v = self._views[i]
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
                self._callback_queued = True
            b = self._bucket_of[i]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
                self._launch_ready()
        return hook

    def _launch_ready(self) -> None:
        for b in self.buckets:
            if self._launched[b.index]:
                continue
            if not self._ready[b.index]:
                break  # keep identical launch order across ranks
            view = self.flat_grad[b.offset:b.offset + b.numel]
            if self.flat_comm is not None:
                wire = self.flat_comm[b.offset:b.offset + b.numel]
                _cast(view, wire)  # on the compute stream: the comm stream's fork orders it
                self._handles.append(self.comm.all_reduce_avg(wire, async_op=True))
                self._casts.append((wire, view))
            else:
                self._handles.append(self.comm.all_reduce_avg(view, async_op=True))
            self._launched[b.index] = True

    def _finalize(self) -> None:
        if not all(self._launched):
            missing = [b.index for b in self.buckets if not self._launched[b.index]]
            self._reset_counts()
            raise RuntimeError(f"DDP: buckets {missing} never became ready (unused parameters?)")
        for h in self._handles:
            h.wait()
        for wire, view in self._casts:  # after the join: the averaged bf16 bucket -> fp32 grads
            _cast(wire, view)
        self._casts = []
        self._reset_counts()

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if self.training and torch.is_grad_enabled():
            if self.broadcast_buffers:
                self._sync_buffers()
            self._attach_grad_views(zero=True)
            self._buffers_synced_for_eval = False
        elif self.broadcast_buffers and not self._buffers_synced_for_eval:
            self._sync_buffers()
            self._buffers_synced_for_eval = True
        return self.module(*args, **kwargs)

    def zero_grad(self, set_to_none: bool = True) -> None:  # keep grads as bucket views
        self.flat_grad.zero_()

    def bucket_sizes_mib(self) -> List[float]:
        return [b.nbytes / (1024 * 1024) for b in self.buckets]

    def bucket_param_names(self) -> List[List[str]]:
        return [[self._names[i] for i in b.param_indices] for b in self.buckets]
