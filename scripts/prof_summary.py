#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (.db from --kernel-trace, or *kernel_trace.csv) into a
per-kernel stats table (calls, total/avg us, share) — the file committed under profiles/."""
import argparse
import collections
import csv
import glob
import os
import sqlite3


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select s.display_name, d.start, d.end, d.grid_size_x, d.grid_size_y, d.grid_size_z, "
         "d.workgroup_size_x, s.arch_vgpr_count, s.accum_vgpr_count, s.group_segment_size "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
    for r in c.execute(q):
        yield {"name": r[0], "start": r[1], "end": r[2], "grid": (r[3], r[4], r[5]), "wg": r[6],
               "vgpr": r[7], "agpr": r[8], "lds": r[9]}


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield {"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                   "grid": (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                   "wg": r.get("Workgroup_Size_X"), "vgpr": r.get("VGPR_Count"), "agpr": r.get("Accum_VGPR_Count"),
                   "lds": r.get("LDS_Block_Size")}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path", help="rocprofv3 output dir or file")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--skip-first", type=float, default=0.0, help="drop dispatches in the first X fraction of time")
    p.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    p.add_argument("--timeline", type=int, default=0, help="also print the last N dispatches in order (one step)")
    a = p.parse_args()
    files = [a.path] if os.path.isfile(a.path) else (glob.glob(os.path.join(a.path, "**", "*.db"), recursive=True) or
                                                     glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                               recursive=True))
    rows = []
    for f in files:
        rows += list(rows_from_db(f) if f.endswith(".db") else rows_from_csv(f))
    rows.sort(key=lambda r: r["start"])
    if a.skip_first and rows:
        t0, t1 = rows[0]["start"], rows[-1]["end"]
        cut = t0 + a.skip_first * (t1 - t0)
        rows = [r for r in rows if r["start"] >= cut]
    agg = collections.OrderedDict()
    meta = {}
    for r in rows:
        d = (r["end"] - r["start"]) / 1e3
        k = r["name"]
        e = agg.setdefault(k, [0, 0.0, 1e30, 0.0])
        e[0] += 1
        e[1] += d
        e[2] = min(e[2], d)
        e[3] = max(e[3], d)
        meta[k] = r
    total = sum(e[1] for e in agg.values())
    span = (rows[-1]["end"] - rows[0]["start"]) / 1e3 if rows else 0.0
    print(f"# {len(rows)} dispatches, kernel time {total:.1f} us, wall span {span:.1f} us"
          + (f", per step: kernel {total / a.steps:.1f} us, span {span / a.steps:.1f} us" if a.steps else ""))
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'pct':>6s}"
          f"  grid / wg / vgpr+agpr / lds")
    for k, e in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        m = meta[k]
        print(f"{k[:70]:70s} {e[0]:6d} {e[1]:10.1f} {e[1] / e[0]:9.2f} {e[2]:8.2f} {e[3]:8.2f} {100 * e[1] / total:6.2f}"
              f"  {m['grid']} / {m['wg']} / {m['vgpr']}+{m['agpr']} / {m['lds']}")
    if a.timeline and rows:
        tl = rows[-a.timeline:]
        print(f"\n# timeline of the last {len(tl)} dispatches: start offset / duration / gap to previous end (us)")
        prev = None
        for r in tl:
            gap = (r["start"] - prev) / 1e3 if prev is not None else 0.0
            print(f"{(r['start'] - tl[0]['start']) / 1e3:9.1f} {(r['end'] - r['start']) / 1e3:8.2f} {gap:7.2f}  "
                  f"{r['name'][:60]}  {r['grid']}")
            prev = r["end"]


if __name__ == "__main__":
    main()
