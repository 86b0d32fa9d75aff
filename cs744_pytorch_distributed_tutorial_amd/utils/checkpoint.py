"""Checkpoint / resume.

The reference never saves anything; its de-facto layout is the VGG ``state_dict``
(58 keys for VGG-11, §2.6). A checkpoint here is a ``torch.save`` dict::

    {"model": <state_dict, no "module." prefix — loadable into the reference _VGG>,
     "optimizer": <torch.optim.SGD state_dict format: momentum_buffer per param
                   index 0..33, param_groups lr/momentum/dampening/wd/nesterov>,
     "epoch": int, "iter": int, "sampler_seed": int, "world_size": int,
     "format": "cs744-amd/1"}

Rank 0 writes (atomically: temp file + rename); every rank loads with
``weights_only=True`` (no pickle code execution) and then the replicas are made
identical by a broadcast from rank 0.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch
import torch.nn as nn

FORMAT = "cs744-amd/1"


def unwrap(model: nn.Module) -> nn.Module:
    return getattr(model, "module", model)


def strip_module_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}


def save_checkpoint(path: str, model_state: Dict[str, torch.Tensor], optimizer_state: Optional[dict] = None,
                    epoch: int = 0, iteration: int = 0, sampler_seed: int = 0, world_size: int = 1,
                    rank: int = 0, extra: Optional[dict] = None) -> None:
    if rank != 0:
        return
    state = {
        "model": {k: v.detach().cpu() for k, v in strip_module_prefix(model_state).items()},
        "optimizer": _to_cpu(optimizer_state) if optimizer_state is not None else None,
        "epoch": int(epoch), "iter": int(iteration), "sampler_seed": int(sampler_seed),
        "world_size": int(world_size), "format": FORMAT,
    }
    if extra:
        state["extra"] = extra
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    state = torch.load(path, map_location=map_location, weights_only=True)
    if not isinstance(state, dict) or "model" not in state:
        raise ValueError(f"{path}: not a cs744-amd checkpoint")
    state["model"] = strip_module_prefix(state["model"])
    return state


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


def save_training_state(path: str, model: nn.Module, optimizer: Optional[torch.optim.Optimizer], epoch: int,
                        iteration: int, sampler_seed: int = 0, world_size: int = 1, rank: int = 0) -> None:
    save_checkpoint(path, unwrap(model).state_dict(), optimizer.state_dict() if optimizer is not None else None,
                    epoch, iteration, sampler_seed, world_size, rank)


def load_training_state(path: str, model: nn.Module, optimizer: Optional[torch.optim.Optimizer] = None,
                        broadcast: bool = True) -> Dict[str, Any]:
    state = load_checkpoint(path)
    m = unwrap(model)
    dev = next(m.parameters()).device
    m.load_state_dict({k: v.to(dev) for k, v in state["model"].items()})
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if broadcast:
        from .. import distributed as D
        if D.get_world_size() > 1:
            for t in list(m.parameters()) + list(m.buffers()):
                D.broadcast(t.data, src=0)
            if optimizer is not None:
                for st in optimizer.state.values():
                    buf = st.get("momentum_buffer")
                    if buf is not None:
                        D.broadcast(buf, src=0)
    return state
