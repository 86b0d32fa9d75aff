"""One tiny forward+backward of VGG-11 through the native HIP path (driver smoke test)."""
from __future__ import annotations

import torch


def run_smoke(device: torch.device, batch: int = 8) -> dict:
    from ..ops import native
    from ..models import VGG11
    from ..utils import data as dm
    C = native.C()  # fails loudly if the extension is missing
    torch.manual_seed(0)
    ds = dm.SyntheticCIFAR10(train=True, size=64, seed=0)
    data = ds.data.to(device)
    idx = torch.arange(batch, device=device)
    params = dm.augment_params(len(ds), 0, 0, True).to(device)
    x = native.augment(data, idx, params, False, 3)
    y = ds.targets[:batch].to(device)
    model = VGG11().to(device)
    try:
        model.native = True
        feat = model(x)
    except NotImplementedError:
        model.native = False
        feat = model(x)
    loss = torch.nn.functional.cross_entropy(feat, y)
    loss.backward()
    g = sum(float(p.grad.abs().sum()) for p in model.parameters())
    torch.cuda.synchronize()
    out = {"loss": float(loss), "grad_l1": g, "native_module": bool(model.native)}
    if not (out["loss"] == out["loss"] and g == g and g > 0):
        raise RuntimeError(f"smoke failed: {out}")
    print(f"[smoke] {out}")
    return out
