"""Ordering check, repeated in one process: the data-parallel step over a one-rank scrambling probe
communicator vs the world-1 step (tests/test_native_distributed_gpu.py::_probe_run), N times;
prints per run whether params / mom / bufs / nbt match bit for bit and, where not, which blocks'
parameters differ (element ranges of the flat layout) and by how much.

    python3 scripts/probe_repeat.py [--runs 4] [--probe order] [--spin 40]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cs744_pytorch_distributed_tutorial_amd as pkg  # noqa: E402

pkg.ensure_hw_queues()
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--runs", type=int, default=4)
    p.add_argument("--probe", default="order")
    p.add_argument("--spin", type=float, default=40.0)
    p.add_argument("--steps", type=int, default=6)
    a = p.parse_args()
    from test_native_distributed_gpu import _probe_run
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    base, _ = _probe_run("0", steps=a.steps)
    for r in range(a.runs):
        out, calls = _probe_run(a.probe, steps=a.steps, spin_us=a.spin)
        rec = {"run": r, "calls": calls}
        for k in base:
            eq = torch.equal(base[k], out[k])
            rec[k] = eq
            if not eq and k == "params":
                d = (base[k] - out[k]).abs()
                bad = [n for n in lay.param_names if not torch.equal(lay.view(base[k], n), lay.view(out[k], n))]
                rec["params_diff"] = {"max_abs": float(d.max()), "n": int((d > 0).sum()), "tensors": bad[:12]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
