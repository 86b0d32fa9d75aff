"""Failure detection and fault injection.

The reference has none: it relies on gloo's 30-minute default timeout and ships
a latent hang (the unmatched accuracy ``isend``, `slave/part2b/part2b.py:68-69`).
This module provides:

* ``CS744_FAULT="<op>:<rank>:<action>[:<arg>]"`` fault injection, consulted by
  every facade collective (`distributed._fault_hook`). Actions: ``kill`` (exit the
  rank with code 17), ``delay`` (sleep ``arg`` seconds), ``raise`` (RuntimeError).
  ``<op>`` may be ``*``; ``<rank>`` may be ``*``; an optional ``@N`` suffix on the
  op fires only at the N-th call (``all_reduce@3:1:kill``).
* ``check_finite`` — NaN/Inf guard on gradients (debug mode).
* ``param_checksum`` / ``assert_replicas_in_sync`` — a cross-rank checksum
  all-gather that catches a missed/mismatched collective (every K steps).
* ``Watchdog`` — a host thread that aborts the process when a step exceeds a
  deadline (a collective hang turns into a loud failure instead of a silent stall).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Dict, Iterable, Optional

import torch

_calls: Dict[str, int] = {}


def _parse(spec: str):
    parts = spec.split(":")
    if len(parts) < 3:
        raise ValueError(f"bad CS744_FAULT spec {spec!r}")
    op, rank, action = parts[0], parts[1], parts[2]
    arg = parts[3] if len(parts) > 3 else None
    nth = None
    if "@" in op:
        op, n = op.split("@", 1)
        nth = int(n)
    return op, rank, action, arg, nth


def maybe_inject(op_name: str, rank: int) -> None:
    spec = os.environ.get("CS744_FAULT")
    if not spec:
        return
    for one in spec.split(","):
        op, r, action, arg, nth = _parse(one)
        if op not in ("*", op_name) or r not in ("*", str(rank)):
            continue
        key = f"{op}:{r}"
        _calls[key] = _calls.get(key, 0) + 1
        if nth is not None and _calls[key] != nth:
            continue
        if action == "kill":
            sys.stderr.write(f"[fault] rank {rank}: killing at {op_name}\n")
            sys.stderr.flush()
            os._exit(17)
        elif action == "delay":
            time.sleep(float(arg or 1.0))
        elif action == "raise":
            raise RuntimeError(f"[fault] injected failure at {op_name} on rank {rank}")
        else:
            raise ValueError(f"unknown fault action {action!r}")


def check_finite(tensors: Iterable[torch.Tensor], what: str = "grad") -> None:
    for i, t in enumerate(tensors):
        if t is not None and not torch.isfinite(t).all():
            raise FloatingPointError(f"non-finite {what} in tensor #{i} (shape {tuple(t.shape)})")


def param_checksum(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    """Order-sensitive float64 checksum of a list of tensors (on their device)."""
    acc = None
    for i, t in enumerate(tensors):
        v = t.detach().double()
        s = v.sum() + (i + 1) * 1e-3 * v.abs().sum()
        acc = s if acc is None else acc + s
    if acc is None:
        return torch.zeros((), dtype=torch.float64)
    return acc.reshape(1)


def assert_replicas_in_sync(tensors: Iterable[torch.Tensor], rtol: float = 0.0, atol: float = 0.0) -> float:
    """All-gather a checksum and raise if ranks disagree; returns the spread."""
    from .. import distributed as D
    cs = param_checksum(list(tensors))
    ws = D.get_world_size()
    if ws == 1:
        return 0.0
    dev = D.device() if D.get_backend() == "nccl" else torch.device("cpu")
    cs = cs.to(dev)
    out = [torch.zeros_like(cs) for _ in range(ws)]
    D.all_gather(out, cs)
    vals = torch.cat(out).cpu()
    spread = float(vals.max() - vals.min())
    if spread > atol + rtol * float(vals.abs().max()):
        raise RuntimeError(f"replicas diverged: checksums {vals.tolist()} (spread {spread:.3e})")
    return spread


class Watchdog:
    """Abort the process if ``kick()`` is not called within ``timeout_s``.

    ``on_timeout`` runs first (the native trainers pass their communicator's abort —
    ``ncclCommAbort`` unblocks RCCL kernels spinning on a dead peer), then the process
    exits with code 18: a hung collective becomes a prompt, loud failure instead of the
    reference's silent 30-minute gloo stall (`master/part2a/part2a.py:84`)."""

    def __init__(self, timeout_s: float, what: str = "step", on_timeout=None):
        self.timeout_s, self.what = timeout_s, what
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "Watchdog":
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def kick(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            if time.monotonic() - self._last > self.timeout_s:
                sys.stderr.write(f"[watchdog] {self.what} exceeded {self.timeout_s:.1f}s — aborting\n")
                sys.stderr.flush()
                if self.on_timeout is not None:
                    try:
                        self.on_timeout()
                    except Exception as e:  # noqa: BLE001 - exiting anyway
                        sys.stderr.write(f"[watchdog] abort hook failed: {e}\n")
                os._exit(18)
