"""One tiny training step of VGG-11 through the native engine (driver smoke test):
on-device augmentation -> conv/BN/ReLU/pool forward -> fused linear+xent ->
hand-scheduled backward -> fused SGD, every op a gfx950 kernel from ``_C.so``."""
from __future__ import annotations

import torch


def run_smoke(device: torch.device, batch: int = 8) -> dict:
    from ..ops import native
    from .engine import NativeTrainer
    native.C()  # fails loudly if the extension is missing
    torch.cuda.set_device(device)
    tr = NativeTrainer(batch_size=batch, device=device, train_size=64, test_size=16, autotune=False, graph="none")
    p0 = tr.params.clone()
    tr.step()
    torch.cuda.synchronize()
    loss = tr.last_loss()
    g = float(tr.grads.abs().sum())
    moved = float((tr.params - p0).abs().max())
    out = {"loss": loss, "grad_l1": g, "max_param_update": moved, "engine": "native"}
    if not (loss == loss and g == g and g > 0 and moved > 0):
        raise RuntimeError(f"smoke failed: {out}")
    print(f"[smoke] {out}")
    return out
