"""In-process ablation / A-B of the native VGG step (one process, one trainer, variants interleaved
round by round — cdna_hip_programming.md §5.4 rule 24: cross-process variance looks like a kernel
property). A variant is an engine debug-skip mask (VggEngine::set_debug_skip: the upper bound of
what fusing away a launch class could save — WRONG numbers while set) and/or the serial backward
and/or a conv tile override (TILESETS below; exact numerics, only the kernels change).

    python scripts/ablate.py --variants base no_fwd_apply:mask=4 serial:serial side_small:tiles=wg16 \
        lag3:lag=3,file=scripts/tables/st_co.json --rounds 5 --steps 50
Prints one JSON line per variant: median / min ms per step over the rounds."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cs744_pytorch_distributed_tutorial_amd as pkg  # noqa: E402

pkg.ensure_hw_queues()
import torch  # noqa: E402


X6S, REGS, KG2, KG4 = 16, 0, 3, 4


def _lds_kib(bm, bn, bk, stage, mode):
    """LDS of one conv GEMM block (conv_gemm.hip TileXS / Tile), KiB — for co-residency planning."""
    a_kc = mode in (0, 1)
    b_kc = mode == 0
    if stage & X6S:
        pa = bk + 8 if a_kc else bm + 32
        pb = bk + 8 if b_kc else bn + 32
        la = (bm if a_kc else bk) * pa
        lb = (bn if b_kc else bk) * pb
        return 2 * 3 * (la + lb) * 2 / 1024
    la = bm * (bk + 4) if a_kc else bk * (bm + 4)
    lb = bn * (bk + 4) if b_kc else bk * (bn + 4)
    return 2 * (la + lb) * 4 / 1024


def _wg_small(tr, bk=16, stage=X6S | REGS, min_blocks=256):
    """every weight gradient (blocks >= 1) as 64x64 tiles with a small LDS footprint (bk16 X6S: 37 KiB)
    so a main-stream GEMM block (<= ~110 KiB) can share its CU instead of queueing behind it"""
    for l, (cin, cout, hw) in enumerate(tr._dims):
        if l == 0:
            continue
        M, N, K = cout, 9 * cin, tr.B * hw * hw
        tiles = ((M + 63) // 64) * ((N + 63) // 64)
        ks = (K + bk - 1) // bk
        sp = 1
        while tiles * sp < min_blocks and ks // (2 * sp) >= 8:
            sp *= 2
        tr.engine.set_tile(l, 2, 64, 64, sp, bk, stage)


TILESETS = {
    "wg16": lambda tr: _wg_small(tr, 16, X6S | REGS, 256),
    "wg16x": lambda tr: _wg_small(tr, 16, X6S | REGS, 512),
}


def main() -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--variants", nargs="+", default=["base:0"])
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--model", default="VGG11")
    args = p.parse_args()
    from cs744_pytorch_distributed_tutorial_amd.ops import native
    torch.cuda.set_device(0)
    native.C().reserve_streams()
    from cs744_pytorch_distributed_tutorial_amd.runtime.engine import NativeTrainer
    tr = NativeTrainer(model=args.model, batch_size=args.batch_size, device=torch.device("cuda", 0), graph="none")
    base_overlap = tr.overlap_wgrad
    specs = tr.layout.specs
    tr._dims = [(4 if l == 0 else s.cin, s.cout, s.hw) for l, s in enumerate(specs)]
    shipped = [[l, m] + list(tr.engine.get_tile(l, m)) for l in range(tr.layout.L) for m in range(3)
               if not (l == 0 and m == 1)]
    for t in shipped:
        print(f"[tiles] block {t[0]} mode {t[1]}: {t[2]}x{t[3]} splits {t[4]} bk {t[5]} stage {t[6]} "
              f"lds {_lds_kib(t[2], t[3], t[5], t[6], t[1]):.1f} KiB", file=sys.stderr)

    def apply_tiles(name):
        for t in shipped:  # [block, mode, bm, bn, splits, bk, stage] -> set_tile(block, mode, bm, bn, splits, bk, stage)
            tr.engine.set_tile(t[0], t[1], t[2], t[3], t[4], t[5], t[6])
        if name.startswith("file="):  # a step_tune.py output (tiles [[block, mode, bm, bn, splits, bk, stage]])
            with open(name[5:]) as f:
                for t in json.load(f)["tiles"]:
                    tr.engine.set_tile(*t[:7])
        elif name:
            TILESETS[name](tr)
    variants = []
    for v in args.variants:
        # NAME[:opt,opt,...]  opts: mask=M serial tiles=NAME|file=PATH fused=FWD_T/BWD_P fin stagger lag=N conv0=0|1 fold=0|1 sgdfold=0|1 batchfold=0|1 headfold=0|1 sidetail=0|1 headtail=0|1
        name, _, rest = v.partition(":")
        o = {"mask": 0, "serial": False, "tiles": "", "fused": (0, 0), "fin": False, "stagger": False, "lag": 0,
             "conv0": 1, "fold": 1, "sgdfold": 1, "batchfold": 1, "headfold": 1, "sidetail": 1, "headtail": 0}
        for tok in filter(None, rest.split(",")):
            k, _, val = tok.partition("=")
            if k == "mask":
                o["mask"] = int(val)
            elif k == "tiles":
                o["tiles"] = val
            elif k == "file":
                o["tiles"] = "file=" + val
            elif k == "fused":
                o["fused"] = tuple(int(x) for x in val.split("/"))
            elif k in ("lag", "conv0", "fold", "sgdfold", "batchfold", "headfold", "sidetail", "headtail"):
                o[k] = int(val)
            elif k in ("serial", "fin", "stagger"):
                o[k] = True
            else:
                raise SystemExit(f"unknown variant option {tok!r}")
        variants.append((name, o))
    import gc
    gc.collect()
    gc.disable()
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    # every variant starts from this state: a skip mask leaves stale (or, over many steps, non-finite)
    # activations and weights behind, and degenerate data runs faster (DVFS) — it must not leak into
    # the next variant's timing
    snap = [t.clone() for t in (tr.params, tr.mom, tr.bufs, tr.nbt)]
    cursor = tr.engine.cursor().clone()
    times = {v[0]: [] for v in variants}
    losses = {v[0]: [] for v in variants}
    for _ in range(args.rounds):
        for name, o in variants:
            tr.engine.set_lag(0)  # joins deferred work before the state is restored
            for dst, src in zip((tr.params, tr.mom, tr.bufs, tr.nbt), snap):
                dst.copy_(src)
            tr.engine.cursor().copy_(cursor)
            apply_tiles(o["tiles"])
            tr.engine.set_bn_fused_limits(*o["fused"])
            tr.engine.set_fin(o["fin"])
            tr.engine.set_stagger(o["stagger"])
            tr.engine.set_lag(o["lag"])
            tr.engine.set_conv0_direct(bool(o["conv0"]))
            tr.engine.set_conv0_bn_fold(bool(o["fold"]))
            tr.engine.set_conv0_sgd_fold(bool(o["sgdfold"]))
            tr.engine.set_conv0_batch_fold(bool(o["batchfold"]))
            tr.engine.set_head_bn_fold(bool(o["headfold"]))
            tr.engine.set_side_sgd_tail(bool(o["sidetail"]))
            tr.engine.set_head_tail(bool(o["headtail"]))
            tr.engine.set_debug_skip(o["mask"])
            tr.engine.set_overlap(base_overlap and not o["serial"])
            for _ in range(args.warmup):
                tr.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                tr.step()
            torch.cuda.synchronize()
            times[name].append(1e3 * (time.perf_counter() - t0) / args.steps)
            losses[name].append(tr.last_loss())
    tr.engine.set_debug_skip(0)
    tr.engine.set_lag(0)
    tr.engine.set_overlap(base_overlap)
    base = statistics.median(times[variants[0][0]])
    for name, o in variants:
        med = statistics.median(times[name])
        print(json.dumps({"variant": name, "opts": {k: (list(v) if isinstance(v, tuple) else v) for k, v in o.items()},
                          "ms_median": round(med, 4), "ms_min": round(min(times[name]), 4),
                          "img_s_median": round(args.batch_size * 1e3 / med, 1),
                          "delta_vs_first_pct": round(100.0 * (med - base) / base, 2),
                          "ms_all": [round(t, 4) for t in times[name]],
                          "loss_last": [round(x, 4) for x in losses[name]]}), flush=True)
    tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
