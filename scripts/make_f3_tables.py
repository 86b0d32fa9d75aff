"""Derive the shipped F3 conv tile tables (runtime/tiles_gfx950.json, version v3) from the v2
ones: every X6S split-bf16 GEMM of blocks >= 1 keeps its tile, K-step, split-K and staging and
switches to the F3 math (scaled fp16 hi/lo, 3 MFMAs; conv_gemm.hip). Measured on MI355X,
cross-process, VGG-11 B=64 (profiles/r6_f3_ab.jsonl): the converted table beat the v2 X6S table by
8-9 % per step and tied a fresh per-GEMM autotune with F3 candidates (0.593 vs 0.599 ms), so the
step-tuned v2 tiles are kept. bf16-mode tables (stage 32) are copied unchanged.

    python3 scripts/make_f3_tables.py   (rewrites runtime/tiles_gfx950.json in place)
"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "cs744_pytorch_distributed_tutorial_amd", "runtime", "tiles_gfx950.json")
X6S, F3 = 16, 64


def f3_ok(stage, bm, bn, bk):
    st = stage & ~X6S
    return st in (0, 3, 4) and not (bk == 64 and bm == 128 and bn == 128)


def main():
    with open(PATH) as f:
        db = json.load(f)
    out = dict(db)
    for key, ent in db.items():
        if not key.endswith("/gfx950/v2"):
            continue
        tiles = []
        n = 0
        for t in ent["tiles"]:
            t = list(t)
            l, m, bm, bn, sp, bk = t[:6]
            st = t[6] if len(t) > 6 else 0
            if l >= 1 and st & X6S and f3_ok(st, bm, bn, bk):
                t = [l, m, bm, bn, sp, bk, (st & ~X6S) | F3]
                n += 1
            tiles.append(t)
        new = {"tiles": tiles, "us": ent.get("us"),
               "note": f"v2 tiles with the F3 math on {n} X6S GEMMs (scripts/make_f3_tables.py)"}
        out[key[:-2] + "v3"] = new
    with open(PATH, "w") as f:
        json.dump(out, f, indent=1)
    print("v3 entries:", sorted(k for k in out if k.endswith("/v3")))


if __name__ == "__main__":
    main()
