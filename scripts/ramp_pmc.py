#!/usr/bin/env python3
"""Start-up ramp, counter view: from one rocprofv3 --pmc (+ --kernel-trace) pass over a long run
(scripts/ramp_run.py), per kernel name compare early and late steps (default 5-25 vs 200-220):
duration, GRBM_GUI_ACTIVE (GPU-busy cycles, summed over the 8 XCDs) and SQ_BUSY_CYCLES, and the
effective clock GRBM_GUI_ACTIVE / 8 / duration. Same cycles at a lower clock = power / data
toggling; more cycles = a data-dependent code path.

    python3 scripts/ramp_pmc.py gpurun_out/ramp_pmc --steps 230
"""
import argparse
import collections
import csv
import glob
import os


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--steps", type=int, default=230)
    p.add_argument("--early", default="5:25")
    p.add_argument("--late", default="200:220")
    a = p.parse_args()
    ctr = collections.defaultdict(dict)  # dispatch id -> counter -> value
    name = {}
    for f in glob.glob(os.path.join(a.path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                d = int(r["Dispatch_Id"])
                ctr[d][r["Counter_Name"]] = ctr[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                name[d] = r.get("Kernel_Name", "?")
    dur = {}
    for f in glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    by = collections.defaultdict(list)
    for d in sorted(ctr):
        by[name[d]].append(d)
    e0, e1 = (int(x) for x in a.early.split(":"))
    l0, l1 = (int(x) for x in a.late.split(":"))
    print(f"# per kernel: early steps {a.early} vs late {a.late}; clock = GRBM_GUI_ACTIVE / 8 / duration")
    print(f"{'kernel':58s} {'n/st':>4s} {'dur_e':>7s} {'dur_l':>7s} {'gui_e':>9s} {'gui_l':>9s} {'busy_e':>9s} "
          f"{'busy_l':>9s} {'MHz_e':>6s} {'MHz_l':>6s}")
    rows = []
    for k, ds in by.items():
        per = len(ds) / a.steps
        if per < 0.99 or not ds:
            continue
        per_i = max(1, round(per))

        def mean(sel, key):
            v = [ctr[d].get(key, 0.0) if key != "dur" else dur.get(d, float("nan")) for d in sel]
            v = [x for x in v if x == x]
            return sum(v) / len(v) if v else float("nan")
        early = ds[e0 * per_i:e1 * per_i]
        late = ds[l0 * per_i:l1 * per_i]
        de, dl = mean(early, "dur"), mean(late, "dur")
        ge, gl = mean(early, "GRBM_GUI_ACTIVE"), mean(late, "GRBM_GUI_ACTIVE")
        be, bl = mean(early, "SQ_BUSY_CYCLES"), mean(late, "SQ_BUSY_CYCLES")
        rows.append((de * per_i - dl * per_i, k, per_i, de, dl, ge, gl, be, bl))
    for delta, k, per_i, de, dl, ge, gl, be, bl in sorted(rows, reverse=True):
        mhz = lambda g, d: g / 8 / d if d == d and d > 0 else float("nan")  # noqa: E731  cycles / us = MHz
        n = k.replace("(anonymous namespace)::", "").replace("void ", "")[:58]
        print(f"{n:58s} {per_i:4d} {de:7.2f} {dl:7.2f} {ge:9.0f} {gl:9.0f} {be:9.0f} {bl:9.0f} {mhz(ge, de):6.0f} "
              f"{mhz(gl, dl):6.0f}")


if __name__ == "__main__":
    main()
