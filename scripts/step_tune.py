"""Step-level conv tile tuning of the native VGG engine (one MI355X).

The engine's own autotune (VggEngine::autotune) times every conv GEMM ALONE. In the real step the
weight gradients run on a side stream next to the main chain's data gradients and BatchNorm
kernels, so a GEMM's cost to the step depends on what it shares the chip with: a side block that
holds 120 KiB of a CU's 160 KiB LDS keeps a main-stream block off that CU until it retires
(profiles/r5_ablate_*.txt). This tuner ranks tiles by what they do to the WHOLE step:

  1. per GEMM, time every valid fp32-accurate candidate alone (X6S split-bf16 maths, register or
     K-group staging; conv0's forward keeps the exact f32 kernel) and keep the fastest few, plus
     the fastest few small-LDS ones (<= --small-lds KiB: they can share a CU with a main block);
  2. coordinate descent on the measured step time: GEMMs in decreasing isolated time, each
     candidate in place in the live step, the best re-checked against the incumbent in interleaved
     rounds and kept only if it wins by > --min-gain percent.

Every candidate is a kernel the GPU test-suite holds to 2e-5 relative against f64, so a table from
here changes speed, not numerics. Output: one JSON object, a drop-in entry for
runtime/tiles_gfx950.json ({"tiles": [[block, mode, bm, bn, splits, bk, stage], ...], "us": ...}).

    python scripts/step_tune.py --out gpurun_out/step_tune.json
    python scripts/step_tune.py --probe xgmi:150:8:25:16 --out gpurun_out/step_tune_dp.json   # N>1 table

N>1 (--probe): RCCL runs each collective as CTAs that occupy CUs while the backward GEMMs run. A
tile whose grid is exactly one 1024-thread block per CU then needs a second wave for the blocks
whose CU an RCCL CTA holds (the one-GPU projection saw 0.69 -> 1.02 ms per step from 16 busy
CTAs), so the data-parallel step gets its own table, tuned with the communicator model running.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import cs744_pytorch_distributed_tutorial_amd as pkg  # noqa: E402

pkg.ensure_hw_queues()
import torch  # noqa: E402

from ablate import _lds_kib  # noqa: E402

X6S = 16
STAGES = (X6S | 0, X6S | 3, X6S | 4)  # X6S register staging, K-groups of 2 / 4
SPLITS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 128, 256)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def candidates(tr, l, mode):
    cin, cout, hw = tr._dims[l]
    B = tr.B
    M, N, K = ((B * hw * hw, cout, 9 * cin) if mode == 0 else (B * hw * hw, cin, 9 * cout) if mode == 1
               else (cout, 9 * cin, B * hw * hw))
    out = []
    conv0_fwd = l == 0 and mode == 0
    stages = (0,) if conv0_fwd else STAGES
    for st in stages:
        for bk in ((16, 32) if conv0_fwd else (16, 32, 64)):
            for bm in (64, 128):
                for bn in (64, 128):
                    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
                    ks = (K + bk - 1) // bk
                    seen = set()
                    for sp in SPLITS:
                        if sp > 1 and ks // sp < 2:
                            continue
                        per = (ks + sp - 1) // sp
                        eff = (ks + per - 1) // per
                        blocks = tiles * eff
                        if eff in seen or blocks > 2048 or (blocks < 64 and eff < ks // 2):
                            continue
                        seen.add(eff)
                        out.append((bm, bn, sp, bk, st))
    return out


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--model", default="VGG11")
    p.add_argument("--keep", type=int, default=5, help="fastest-alone candidates kept per GEMM")
    p.add_argument("--keep-small", type=int, default=3, help="fastest small-LDS candidates kept per GEMM")
    p.add_argument("--small-lds", type=float, default=75.0)
    p.add_argument("--steps", type=int, default=40, help="timed steps per in-step measurement")
    p.add_argument("--verify-rounds", type=int, default=3)
    p.add_argument("--min-gain", type=float, default=0.3, help="percent")
    p.add_argument("--passes", type=int, default=1)
    p.add_argument("--budget-s", type=float, default=900.0)
    p.add_argument("--out", default=None)
    p.add_argument("--start", default="shipped",
                   help="shipped | coresident (every GEMM at its fastest-alone tile within --co-lds-main / "
                        "--co-lds-side KiB, so a main-stream and a side-stream block fit one CU together) | "
                        "file:PATH (a previous step_tune.py output)")
    p.add_argument("--lag", type=int, default=None, help="engine set_lag(N) during the tuning (default: engine default)")
    p.add_argument("--probe", default=None,
                   help="tune under a one-GPU communicator model, e.g. xgmi:150:8:25:16 (N=8 ring at 150 GB/s, "
                        "16 busy CTAs per collective: the N>1 table, runtime/tiles_gfx950.json key '.../dp')")
    p.add_argument("--co-lds-main", type=float, default=80.0)
    p.add_argument("--co-lds-side", type=float, default=75.0)
    args = p.parse_args()
    t_start = time.time()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(model=args.model, batch_size=args.batch_size, device=torch.device("cuda", 0), graph="none",
                       probe=args.probe)
    tr._dims = [(4 if l == 0 else s.cin, s.cout, s.hw) for l, s in enumerate(tr.layout.specs)]
    eng = tr.engine
    if args.lag is not None:
        eng.set_lag(args.lag)
    gemms = [(l, m) for l in range(tr.layout.L) for m in range(3) if not (l == 0 and m == 1)]
    cur = {g: list(eng.get_tile(*g)) for g in gemms}  # [bm, bn, splits, bk, stage]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def set_t(g, t):
        eng.set_tile(g[0], g[1], t[0], t[1], t[2], t[3], t[4])

    def alone(g, t, reps=6):
        set_t(g, t)
        eng.run_conv(g[0], g[1], tr.B)
        e0.record()
        for _ in range(reps):
            eng.run_conv(g[0], g[1], tr.B)
        e1.record()
        e1.synchronize()
        return 1e3 * e0.elapsed_time(e1) / reps

    def step_ms(n=None):
        n = n or args.steps
        for _ in range(4):
            tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            tr.step()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    import gc
    gc.collect()
    gc.disable()
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    if args.start.startswith("file:"):
        with open(args.start[5:]) as f:
            for t in json.load(f)["tiles"]:
                cur[(t[0], t[1])] = list(t[2:7])
    eng.join_lag()  # isolated timings write gradients the deferred SGD would read
    torch.cuda.synchronize()
    # ---- phase 1: isolated timings
    short = {}
    iso_cur = {}
    for g in gemms:
        res = []
        for t in candidates(tr, *g):
            try:
                res.append((alone(g, t), t))
            except RuntimeError:
                continue
        res.sort(key=lambda x: x[0])
        if args.start == "coresident":
            cap = args.co_lds_side if g[1] == 2 else args.co_lds_main
            fit = [t for _, t in res if _lds_kib(t[0], t[1], t[3], t[4], g[1]) <= cap]
            if fit and not (g[0] == 0 and g[1] == 0):
                cur[g] = list(fit[0])
        set_t(g, cur[g])
        iso_cur[g] = alone(g, cur[g])
        set_t(g, cur[g])
        keep = [t for _, t in res[:args.keep]]
        small = [t for us, t in res if _lds_kib(t[0], t[1], t[3], t[4], g[1]) <= args.small_lds][:args.keep_small]
        short[g] = [list(t) for t in dict.fromkeys(tuple(t) for t in keep + small) if list(t) != cur[g]]
        log(f"[alone] {g}: current {cur[g]} {iso_cur[g]:.1f} us; best alone {res[0][1]} {res[0][0]:.1f} us; "
            f"{len(res)} valid, {len(short[g])} kept")
    # ---- phase 2: coordinate descent on the step time
    base = statistics.median(step_ms() for _ in range(3))
    log(f"[step] start {base:.4f} ms")
    order = sorted(gemms, key=lambda g: -iso_cur[g])
    history = []
    for ps in range(args.passes):
        for g in order:
            if time.time() - t_start > args.budget_s:
                log("[step] time budget reached")
                break
            best_t, best_ms = None, None
            ref = step_ms()
            for t in short[g]:
                set_t(g, t)
                ms = step_ms()
                if best_ms is None or ms < best_ms:
                    best_t, best_ms = t, ms
            set_t(g, cur[g])
            if best_t is None or best_ms >= ref:
                continue
            # interleaved verification: incumbent vs challenger
            a, b = [], []
            for _ in range(args.verify_rounds):
                set_t(g, cur[g])
                a.append(step_ms(2 * args.steps))
                set_t(g, best_t)
                b.append(step_ms(2 * args.steps))
            gain = 100.0 * (statistics.median(a) - statistics.median(b)) / statistics.median(a)
            if gain > args.min_gain:
                log(f"[step] pass {ps} {g}: {cur[g]} -> {best_t}  {statistics.median(a):.4f} -> "
                    f"{statistics.median(b):.4f} ms ({gain:+.2f} %)")
                history.append({"gemm": list(g), "from": cur[g], "to": best_t, "gain_pct": round(gain, 3)})
                cur[g] = best_t
            else:
                log(f"[step] pass {ps} {g}: kept {cur[g]} (challenger {best_t}: {gain:+.2f} %)")
            set_t(g, cur[g])
    final = statistics.median(step_ms(2 * args.steps) for _ in range(3))
    log(f"[step] end {final:.4f} ms (start {base:.4f})")
    us = []
    for l in range(tr.layout.L):
        for m in range(3):
            us.append(0.0 if (l == 0 and m == 1) else round(alone((l, m), cur[(l, m)]), 3))
            if not (l == 0 and m == 1):
                set_t((l, m), cur[(l, m)])
    ent = {"tiles": [[g[0], g[1]] + cur[g] for g in gemms], "us": us,
           "dual": [0] * tr.layout.L, "step_ms": {"start": round(base, 4), "end": round(final, 4)},
           "history": history, "tuner": "scripts/step_tune.py", "lag": args.lag, "probe": args.probe}
    print(json.dumps(ent), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(ent, f, indent=1)
    tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
