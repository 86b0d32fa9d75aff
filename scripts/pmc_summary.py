#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter CSVs (one dir per pass) plus derived
MFMA utilisation / wait shares — the table committed under profiles/."""
import collections
import csv
import glob
import os
import sys


def load(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "?")
                key = (name, r.get("Dispatch_Id"))
                out[name][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[key] += 1
    disp = collections.Counter(k[0] for k in cnt)
    return out, disp


def short(n, w=60):
    n = n.replace("(anonymous namespace)::", "")
    return n[:w]


def main():
    agg = collections.defaultdict(dict)
    ndisp = {}
    for d in sys.argv[1:]:
        vals, disp = load(d)
        for k, v in vals.items():
            for c, x in v.items():
                agg[k][c] = x / max(disp[k], 1)
            ndisp[k] = disp[k]
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0) * ndisp.get(kv[0], 1))
    print(f"{'kernel':60s} {'n':>4s} {'mfma%':>6s} {'wait%':>6s} {'winst%':>6s} {'active%':>7s} {'ldsconf/lds':>11s} {'L2hit%':>6s}")
    for k, v in rows:
        busy = v.get("SQ_BUSY_CYCLES", 0)
        wc = v.get("SQ_WAVE_CYCLES", 0) or 1
        mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        # SQ_BUSY_CYCLES is per SE aggregate; MFMA busy is summed over SIMDs: report the ratio to GRBM time x 1024 SIMDs
        gui = v.get("GRBM_GUI_ACTIVE", 0)
        mfma = 100.0 * mf / (gui * 128) if gui else float("nan")  # GRBM counts are summed over 8 XCDs; 1024 SIMDs
        hit = v.get("TCC_HIT_sum", 0); miss = v.get("TCC_MISS_sum", 0)
        l2 = 100.0 * hit / (hit + miss) if hit + miss else float("nan")
        lds = v.get("SQ_INSTS_LDS", 0)
        conf = v.get("SQ_LDS_BANK_CONFLICT", 0) / lds if lds else float("nan")
        print(f"{short(k):60s} {ndisp.get(k,0):4d} {mfma:6.1f} {100*v.get('SQ_WAIT_ANY',0)/wc:6.1f} "
              f"{100*v.get('SQ_WAIT_INST_ANY',0)/wc:6.1f} {100*v.get('SQ_ACTIVE_INST_ANY',0)/wc:7.1f} {conf:11.2f} {l2:6.1f}")
    mix = [(k, v) for k, v in rows if v.get("SQ_INSTS_MFMA", 0) > 0]
    if mix:
        # instruction mix per MFMA (F3 issues 3 MFMAs per 32x32x16 product step, X6S 6: compare the
        # per-dispatch VALU count too, not only the ratio)
        print()
        print(f"{'kernel':60s} {'n':>4s} {'mfma%':>6s} {'valu/mfma':>9s} {'lds/mfma':>8s} {'vmem/mfma':>9s} "
              f"{'waitLDS%':>8s} {'kVALU/disp':>10s} {'kMFMA/disp':>10s}")
        for k, v in mix:
            mf = v["SQ_INSTS_MFMA"]
            gui = v.get("GRBM_GUI_ACTIVE", 0)
            util = 100.0 * v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * 128) if gui else float("nan")
            wc = v.get("SQ_WAVE_CYCLES", 0) or 1
            print(f"{short(k):60s} {ndisp.get(k, 0):4d} {util:6.1f} {v.get('SQ_INSTS_VALU', 0) / mf:9.2f} "
                  f"{v.get('SQ_INSTS_LDS', 0) / mf:8.2f} {v.get('SQ_INSTS_VMEM_RD', 0) / mf:9.2f} "
                  f"{100 * v.get('SQ_WAIT_INST_LDS', 0) / wc:8.1f} {v.get('SQ_INSTS_VALU', 0) / 1e3:10.1f} {mf / 1e3:10.1f}")
    print()
    print("raw per-dispatch averages:")
    for k, v in rows[:12]:
        print(short(k, 90), {c: round(x) for c, x in sorted(v.items())})


if __name__ == "__main__":
    main()
