"""Tune the conv tile tables shipped in runtime/tiles_gfx950.json (GPU box):
    CS744_TUNE=1 CS744_TUNE_CACHE=gpurun_out/tiles_gfx950.json python scripts/make_tile_table.py
then copy the JSON into cs744_pytorch_distributed_tutorial_amd/runtime/."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer  # noqa: E402

CONFIGS = [("VGG11", 64, "fp32"), ("VGG11", 128, "fp32"), ("VGG11", 256, "fp32"), ("VGG11", 64, "bf16"),
           ("VGG11", 256, "bf16"), ("VGG13", 64, "fp32"), ("VGG16", 64, "fp32"), ("VGG19", 64, "fp32")]

if __name__ == "__main__":
    assert os.environ.get("CS744_TUNE") == "1" and os.environ.get("CS744_TUNE_CACHE")
    for model, B, dt in CONFIGS:
        t0 = time.time()
        tr = NativeTrainer(model=model, batch_size=B, device=torch.device("cuda", 0), train_size=4096,
                           test_size=64, dtype=dt)
        print(f"{model} B{B} {dt}: {tr.tile_source}, {sum(tr.tune_us):.1f} us of conv GEMMs, "
              f"{time.time() - t0:.1f} s", flush=True)
        tr.close()
