"""A long native-engine run for the start-up ramp analysis (scripts/ramp_table.py): a fresh trainer
at the bench configuration (VGG-11, B = 64, fp32, shipped tiles), N back-to-back steps, no host
syncs inside. Run under rocprofv3 --kernel-trace, or under --pmc for per-dispatch counters.

    python3 scripts/ramp_run.py [--steps 230]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=230)
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(batch_size=64, device=torch.device("cuda", 0))
    import gc
    gc.collect()
    gc.disable()
    torch.cuda.synchronize()
    for i in range(a.steps):
        tr.step()
        if i % 50 == 49:
            print(f"step {i + 1} loss {tr.last_loss():.4f}", flush=True)
    torch.cuda.synchronize()
    tr.close()


if __name__ == "__main__":
    main()
