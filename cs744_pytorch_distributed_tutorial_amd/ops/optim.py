"""Fused multi-tensor SGD (one HIP launch per step for all parameters).

Drop-in for ``torch.optim.SGD(params, lr, momentum, weight_decay)`` as the
reference uses it (`master/part1/part1.py:98-99`): same update rule and same
``state_dict`` format (``momentum_buffer`` per parameter), so checkpoints are
interchangeable. On CPU tensors it defers to torch's implementation.
"""
from __future__ import annotations

import torch

from . import native


_NO_SHADOW = {}


def _shadow_of(p: torch.Tensor) -> torch.Tensor:
    """the live bf16 shadow of ``p`` (registered by ``ops.lm.ShadowLinear``), or an empty tensor"""
    sh = getattr(p, "_cs_bf16_shadow", None)
    if sh is not None and getattr(p, "_cs_bf16_shadow_version", -1) == p._version and sh.numel() == p.numel():
        return sh
    dev = p.device
    if dev not in _NO_SHADOW:
        _NO_SHADOW[dev] = torch.empty(0, device=dev, dtype=torch.bfloat16)
    return _NO_SHADOW[dev]


class FusedSGD(torch.optim.SGD):
    def __init__(self, params, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 grad_scale: float = 1.0):
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov)
        if nesterov:
            raise ValueError("FusedSGD: nesterov not supported (the reference does not use it)")
        self.grad_scale = grad_scale
        self._tables = {}

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            if not ps[0].is_cuda:
                return super().step()
            mom = group["momentum"]
            first = False
            bufs = []
            for p in ps:
                st = self.state[p]
                if st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.zeros_like(p)
                    first = True
                bufs.append(st["momentum_buffer"])
            gs = [p.grad for p in ps]
            # a parameter with a live bf16 shadow (ops.lm.ShadowLinear) gets it rewritten by the same pass
            shs = [_shadow_of(p) for p in ps]
            key = tuple((p.data_ptr(), g.data_ptr(), b.data_ptr(), s.data_ptr() if s.numel() else 0)
                        for p, g, b, s in zip(ps, gs, bufs, shs))
            tab = self._tables.get(id(group))
            if tab is None or tab[0] != key:
                t = native.C().sgd_multi_table(ps, gs, bufs, shs)
                nchunks = int(t[-1].item())
                tab = (key, t, nchunks)
                self._tables[id(group)] = tab
            native.C().sgd_multi(tab[1], len(ps), tab[2], group["lr"], mom, group["weight_decay"],
                                 group["dampening"], self.grad_scale, first and mom != 0)
        return loss
