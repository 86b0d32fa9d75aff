"""Start-up ramp, clock view: the shader clock during each step of a fresh training run, measured
inside the concurrent schedule (a one-wave sampler on its own stream, csrc/kernels/clock_probe.hip),
and the step boundaries on the same 100 MHz axis (a stamp kernel ahead of every step). Per step:
device time, mean clock, and cycles = time x clock. Early vs late steps then split the ramp into
"fewer cycles" and "a faster clock".

    python3 scripts/ramp_clock.py [--steps 230] [--early 5:25] [--late 200:220]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

_pkg.ensure_hw_queues()
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=230)
    p.add_argument("--early", default="5:25")
    p.add_argument("--late", default="200:220")
    p.add_argument("--max-samples", type=int, default=1 << 17)
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    C = native.C()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    C.reserve_streams()
    samp_stream = torch.cuda.Stream(dev)
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(batch_size=64, device=dev)
    out = torch.zeros(2 * (a.max_samples + 1), dtype=torch.int64, device=dev)
    stop = torch.zeros(1, dtype=torch.int32, device=dev)
    slots = torch.zeros(a.steps + 1, dtype=torch.int64, device=dev)
    import gc
    gc.collect()
    gc.disable()
    torch.cuda.synchronize()
    C.clock_sampler(out, stop, samp_stream.cuda_stream)
    time.sleep(0.002)
    for i in range(a.steps):
        C.clock_stamp(slots, i)
        tr.step()
    C.clock_stamp(slots, a.steps)
    C.clock_stop(stop)
    torch.cuda.synchronize()
    o = out.view(-1, 2).cpu().tolist()
    n = next((i for i, (r, _) in enumerate(o) if r == 0), len(o))
    real = [r for r, _ in o[:n]]
    clk = [c for _, c in o[:n]]
    st = slots.cpu().tolist()
    if n < 2 or real[0] > st[0] or real[-1] < st[-1]:
        print(json.dumps({"error": "sampler did not cover the run", "samples": n}))
        sys.exit(1)
    import bisect
    rows = []
    for i in range(a.steps):
        j0 = bisect.bisect_left(real, st[i])
        j1 = bisect.bisect_right(real, st[i + 1]) - 1
        us = (st[i + 1] - st[i]) / 100.0
        mhz = 100.0 * (clk[j1] - clk[j0]) / (real[j1] - real[j0]) if j1 > j0 else float("nan")
        rows.append((us, mhz, us * mhz / 1e3, j1 - j0))

    def win(spec):
        lo, hi = (int(x) for x in spec.split(":"))
        sel = [r for r in rows[lo:hi] if r[1] == r[1]]
        k = max(len(sel), 1)
        return [sum(r[c] for r in sel) / k for c in range(3)]
    print("# per 10 steps: device us/step (stamp to stamp), shader clock MHz (sampler), kcycles/step")
    for i0 in range(0, a.steps, 10):
        blk = [r for r in rows[i0:i0 + 10] if r[1] == r[1]]
        if blk:
            print(f"steps {i0:4d}-{i0 + len(rows[i0:i0 + 10]) - 1:4d}  {sum(r[0] for r in blk) / len(blk):8.1f} "
                  f"{sum(r[1] for r in blk) / len(blk):7.0f} {sum(r[2] for r in blk) / len(blk):9.1f}")
    e, l = win(a.early), win(a.late)
    # step_e / step_l = (cycles_e / cycles_l) * (clock_l / clock_e): the two factors of the ramp
    print(json.dumps({"early": a.early, "late": a.late, "us_e": round(e[0], 1), "us_l": round(l[0], 1),
                      "mhz_e": round(e[1], 1), "mhz_l": round(l[1], 1), "kcyc_e": round(e[2], 1),
                      "kcyc_l": round(l[2], 1), "time_ratio": round(e[0] / l[0], 4),
                      "clock_factor": round(l[1] / e[1], 4), "cycle_factor": round(e[2] / l[2], 4),
                      "samples": n, "loss": round(tr.last_loss(), 4)}), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
