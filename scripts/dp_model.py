"""Analytic N-GPU projection of the VGG-11 data-parallel step (a MODEL, not a measurement; runs on CPU).

Inputs: one measured single-GPU step timeline (scripts/step_timeline.py output, e.g.
profiles/r4_step_timeline_fin.txt: every kernel of one step with start and duration) and the
engine's real bucket plan (FlatLayout.plan_buckets, 4 MiB cap). A bucket's gradients are complete
when the weight-gradient GEMM of its lowest block ends; its ring all-reduce then runs on the comm
stream (one collective at a time, in bucket order) for

    t_ar = alpha + 2 (W - 1) / W * bytes / busBW

(xGMI ring all-reduce; alpha = per-collective latency), followed by that bucket's
SGD update (its share of the measured flat SGD time). While a collective runs, its RCCL CTAs hold
`ctas` of the 256 CUs, so compute that overlaps it is stretched by up to 256 / (256 - ctas) (an
upper bound: it assumes the overlapped GEMMs fill every CU). The step ends at the later of the
compute stream and the comm stream's last SGD, plus the measured one-rank plumbing cost
(fork/join links, BN-buffer broadcast; profiles/r2_dp_plumbing.md: 0.786 vs 0.755 ms = 31 us).
Weak scaling (64 images per GPU): projected img/s = W * 64 / t_step.

Usage: python scripts/dp_model.py [--timeline profiles/r4_step_timeline_fin.txt]
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ROW = re.compile(r"^\s+([0-9.]+)\s+([0-9.]+)\s+(-?[0-9.]+)\s+(\S.*)$")


def read_timeline(path):
    rows = []
    for line in open(path):
        m = ROW.match(line)
        if m:
            rows.append((float(m.group(1)), float(m.group(2)), m.group(4)))
    if not rows:
        raise SystemExit(f"no kernel rows in {path}")
    return rows


def wgrad_ends(rows, L):
    """end time of each block's weight-gradient GEMM (MODE 2 conv kernels, backward order L-1..0)"""
    ends = [r[0] + r[1] for r in rows if re.search(r"conv_gemm_kernel<\d+, \d+, 2,", r[2])]
    if len(ends) != L:
        raise SystemExit(f"expected {L} weight-gradient kernels, found {len(ends)}")
    return {L - 1 - i: e for i, e in enumerate(ends)}


def simulate(rows, lows, ranges, ready, W, gbps, alpha, ctas, sgd_us, plumb_us):
    step_end = rows[-1][0] + rows[-1][1]
    total = sum(n for _, n in ranges)
    t_comm = 0.0
    busy = []
    for low, (_, n) in zip(lows, ranges):
        nbytes = 4 * n
        t_ar = alpha + 2.0 * (W - 1) / W * nbytes / (gbps * 1e3)  # us (GB/s = 1e3 bytes/us)
        start = max(ready[low], t_comm)
        busy.append((start, start + t_ar))
        t_comm = start + t_ar + sgd_us * n / total
    # compute stretched where a collective overlaps it (from the first bucket's start to step end)
    overlap = sum(max(0.0, min(e, step_end) - s) for s, e in busy)
    stretch = overlap * (256.0 / (256.0 - ctas) - 1.0)
    compute_end = step_end + stretch
    return max(compute_end, t_comm) + plumb_us, overlap


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--timeline", default="profiles/r4_step_timeline_fin.txt")
    p.add_argument("--gbps", default="100,150,300")
    p.add_argument("--worlds", default="2,4,8")
    p.add_argument("--ctas", default="8,16,32")
    p.add_argument("--alpha-us", type=float, default=25.0)
    p.add_argument("--plumb-us", type=float, default=31.0)
    p.add_argument("--bucket-mb", type=float, default=4.0)
    a = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import FlatLayout
    lay = FlatLayout("VGG11")
    lows, ranges = lay.plan_buckets(a.bucket_mb)
    rows = read_timeline(a.timeline)
    ready = wgrad_ends(rows, lay.L)
    sgd = [r[1] for r in rows if "sgd" in r[2]]
    sgd_us = sum(sgd) if sgd else 5.0
    t1 = rows[-1][0] + rows[-1][1]
    print(json.dumps({"model": "analytic (not measured)", "timeline": a.timeline, "world1_step_us": round(t1, 1),
                      "world1_img_s": round(64 / t1 * 1e6),
                      "buckets_mib": [round(4 * n / 2 ** 20, 2) for _, n in ranges],
                      "bucket_ready_us": [round(ready[l], 1) for l in lows]}))
    for g in [float(x) for x in a.gbps.split(",")]:
        for w in [int(x) for x in a.worlds.split(",")]:
            for c in [int(x) for x in a.ctas.split(",")]:
                t, ov = simulate(rows, lows, ranges, ready, w, g, a.alpha_us, c, sgd_us, a.plumb_us)
                print(json.dumps({"W": w, "busbw_GBps": g, "comm_ctas": c, "step_us": round(t, 1),
                                  "projected_img_s": round(w * 64 / t * 1e6), "efficiency": round(t1 / t, 3),
                                  "overlapped_comm_us": round(ov, 1)}))


if __name__ == "__main__":
    main()
