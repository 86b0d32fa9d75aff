"""Stale-gradient probe (round-2 advisor finding): world-2 gloo all-reduce issued from Python with
side-stream weight gradients, eager steps, bitwise against the serial backward; REPS runs with the
system-scope join off (CS_SYS_JOIN=0) and on. Prints the mismatching tensors per run.
Usage (on the GPU box): python scripts/sys_join_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from mp_util import run_world  # noqa: E402
from test_native_distributed_gpu import _train  # noqa: E402


def main():
    import cs744_pytorch_distributed_tutorial_amd as pkg
    pkg.ensure_hw_queues()
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ser = run_world(_train, 2, "ddp", "none", 6, "torch", 16, False, {"CS_OVERLAP_WGRAD": "0"})
    for sj in ("0", "1"):
        bad = 0
        for i in range(reps):
            o = run_world(_train, 2, "ddp", "none", 6, "torch", 16, False, {"CS_OVERLAP_WGRAD": "force", "CS_SYS_JOIN": sj})
            diff = [(r, k, float((o[r][k] - ser[r][k]).abs().max())) for r in range(2) for k in ("params", "mom")
                    if not torch.equal(o[r][k], ser[r][k])]
            bad += bool(diff)
            print(f"sys_join={sj} run {i}: side={o[0]['wgrad_side']} {'MISMATCH ' + str(diff) if diff else 'bitwise equal'}",
                  flush=True)
        print(f"sys_join={sj}: {bad}/{reps} runs mismatched", flush=True)


if __name__ == "__main__":
    main()
