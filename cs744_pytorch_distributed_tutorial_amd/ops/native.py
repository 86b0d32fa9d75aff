"""Loader for the in-tree native extension (``_C.so``: gfx950 HIP kernels + C++ runtime).

On a GPU machine a missing or stale extension is a hard error (no silent eager
fallback): set ``CS744_ALLOW_NO_NATIVE=1`` to opt out explicitly. Build it with
``python -m cs744_pytorch_distributed_tutorial_amd._build`` (done by
``__graft_entry__.build()``).
"""
from __future__ import annotations

import os

import torch

_C = None
_err = None


def load(required: bool = None):
    global _C, _err
    if _C is not None:
        return _C
    try:
        from .. import _C as mod  # type: ignore
        _C = mod
        return _C
    except ImportError as e:  # pragma: no cover - depends on build state
        _err = e
    if required is None:
        required = torch.cuda.is_available() and os.environ.get("CS744_ALLOW_NO_NATIVE") != "1"
    if required:
        raise RuntimeError(f"native extension _C.so is not built/importable ({_err}); run "
                           "`python -m cs744_pytorch_distributed_tutorial_amd._build`")
    return None


def available() -> bool:
    try:
        return load(required=False) is not None
    except RuntimeError:
        return False


def C():
    return load(required=True)


def augment(data: torch.Tensor, idx: torch.Tensor, params: torch.Tensor, nhwc: bool = False,
            cstride: int = 3) -> torch.Tensor:
    return C().augment(data, idx, params, nhwc, cstride)


def sgd_flat(p, g, m, lr, momentum, weight_decay, dampening=0.0, scale=1.0, first=False) -> None:
    C().sgd_flat(p, g, m, lr, momentum, weight_decay, dampening, scale, first)


def linear_xent(feat, W, bias, labels, gscale=1.0, backward=True):
    return C().linear_xent(feat, W, bias, labels, gscale, backward)


def softmax_xent(logits, labels, gscale=1.0):
    return C().softmax_xent(logits, labels, gscale)
