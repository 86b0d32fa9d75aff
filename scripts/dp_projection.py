"""N>1 projection of the VGG-11 data-parallel step on ONE MI355X (a model, not a measurement of N GPUs).

The native engine runs its real data-parallel schedule — bucket all-reduces forked from the compute
stream as soon as each bucket's gradients exist, each bucket's SGD behind its all-reduce on the
comm stream, the BN-buffer broadcast, the closing join — against a probe communicator
(ProbeComm "xgmi:G:W:us") whose every all-reduce is a spin as long as a W-GPU ring all-reduce of its
bytes at G GB/s bus bandwidth plus a per-call latency: t = us + 2 (W-1)/W * bytes / G. Compute per
GPU is what weak scaling keeps fixed (B = 64 per GPU), so the projected W-GPU throughput is
W * B / t_step. RCCL's CTAs (CS_COMM_CTAS, default 16 of 256 CUs) competing with the backward GEMMs
while a collective runs are priced with --ctas: the modelled collective then runs as that many busy
workgroups (dependent FMA chains) instead of one sleeping wave. Not modelled: rank skew, and the
memory traffic of the real copy-reduce.

CTA budget (--cta-gbps B > 0): RCCL runs a ring collective as one CTA per channel, and a channel's
throughput is bounded by its CTA's copy-reduce rate as well as by the link, so the bus bandwidth a
collective gets with c CTAs is modelled as min(G, c * B) — the CTA count prices both sides: fewer
CTAs leave more CUs to the backward GEMMs but slow the all-reduce. B is an ASSUMPTION (default
10 GB/s per CTA, i.e. 16 CTAs ~ 160 GB/s), not a measurement on an 8-GPU node.

Every configuration (world 1 included) runs --repeats times, the rounds interleaved, and the
median step time is reported with all samples: one run of a configuration can land on a slow
clock phase (a 2x outlier was seen in a single-pass sweep).

Usage (GPU box): python scripts/dp_projection.py [--steps 50] [--gbps 100,150,300] [--worlds 2,4,8] [--repeats 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cs744_pytorch_distributed_tutorial_amd as _pkg  # noqa: E402

# the engine overlaps weight gradients on a side stream next to a communicator only with >= 8 HIP
# hardware queues (bench.py does the same before HIP starts)
_pkg.ensure_hw_queues()
import torch  # noqa: E402


def run(probe, steps, warmup, B=64, bucket_mb=4.0):
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    dev = torch.device("cuda", 0)
    tr = NativeTrainer(batch_size=B, device=dev, probe=probe, graph="none", bucket_mb=bucket_mb)
    for _ in range(warmup):
        tr.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        tr.step()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    ph = tr.phase_breakdown(5)
    buckets = [n * 4 / 2 ** 20 for _, n in tr.bucket_ranges]
    tr.close()
    return ms, ph, buckets


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--gbps", type=str, default="100,150,300")
    p.add_argument("--worlds", type=str, default="2,4,8")
    p.add_argument("--latency-us", type=float, default=25.0)
    p.add_argument("--ctas", type=str, default="0,8,16,32",
                   help="busy workgroups standing in for RCCL's CTAs during each collective (0: one sleeping wave)")
    p.add_argument("--cta-gbps", type=float, default=0.0,
                   help="> 0: per-CTA channel bandwidth (GB/s); busBW = min(G, ctas * this) (a model)")
    p.add_argument("--repeats", type=int, default=3)
    p.add_argument("--bucket-mb", type=float, default=4.0, help="DDP bucket cap (MiB; layer-aligned buckets)")
    a = p.parse_args()
    torch.cuda.set_device(0)
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    native.C().reserve_streams()  # the side stream owns a hardware queue (as in bench.py)
    configs = [(None, None, None, None)]
    for g in [float(x) for x in a.gbps.split(",")]:
        for w in [int(x) for x in a.worlds.split(",")]:
            for c in [int(x) for x in a.ctas.split(",")]:
                ge = min(g, c * a.cta_gbps) if a.cta_gbps > 0 and c > 0 else g
                configs.append((g, w, c, ge))
    samples = [[] for _ in configs]
    for _ in range(a.repeats):
        for i, (g, w, c, ge) in enumerate(configs):
            probe = "0" if g is None else f"xgmi:{ge}:{w}:{a.latency_us}:{c}"
            samples[i].append(run(probe, a.steps, a.warmup, bucket_mb=a.bucket_mb))
            print(f"[projection] {probe}: {samples[i][-1][0]:.4f} ms", file=sys.stderr, flush=True)
    med = statistics.median_low  # an even count keeps the lower middle sample (outliers are slow)
    base = med([ms for ms, _, _ in samples[0]])
    for i, (g, w, c, ge) in enumerate(configs):
        ms = med([m for m, _, _ in samples[i]])
        ms_all = [round(m, 4) for m, _, _ in samples[i]]
        ph = min(samples[i], key=lambda t: abs(t[0] - ms))[1]
        if g is None:
            buckets = samples[i][0][2]
            print(json.dumps({"config": "world 1 (no communicator)", "ms_per_step": round(ms, 4), "ms_all": ms_all,
                              "img_s": round(64 / ms * 1e3), "bucket_mib": [round(b, 2) for b in buckets],
                              "phases_ms": {k: round(v, 4) for k, v in ph.items()}}), flush=True)
            continue
        print(json.dumps({"config": f"projected N={w}, ring busBW {ge:g} GB/s (link {g:g}), "
                                    f"{a.latency_us:g} us/collective, {c} busy CTAs per collective",
                          "model": "busBW=min(link, ctas*cta_gbps)" if a.cta_gbps > 0 else "busBW=link",
                          "ms_per_step": round(ms, 4), "ms_all": ms_all, "projected_img_s": round(w * 64 / ms * 1e3),
                          "per_gpu_img_s": round(64 / ms * 1e3), "efficiency_vs_world1": round(base / ms, 4),
                          "allreduce_wait_ms": round(ph.get("allreduce_wait", 0.0), 4),
                          "phases_ms": {k: round(v, 4) for k, v in ph.items()}}), flush=True)


if __name__ == "__main__":
    main()
