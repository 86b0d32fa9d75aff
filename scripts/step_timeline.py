#!/usr/bin/env python3
"""One training step of a rocprofv3 kernel trace (.db), per HIP queue: every dispatch with its
start / end offset from the step's first kernel, plus per-queue busy time and the critical
(main-queue) idle gaps. A step = [the second-to-last step-head dispatch, the last one): make_batch, or
the conv0 forward when the batch is built inside it (round 5's fold).
With --last K, first a per-step table of the last K steps (span, main-queue busy and idle); run
under scripts/step_trace_ahead.py for steps whose gaps are the schedule's, not the profiled host's.
Usage: python scripts/step_timeline.py <rocprofv3 out dir> [--names 48] [--last 10]"""
import argparse
import collections
import glob
import os
import sqlite3


def load(path):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]:
        c = sqlite3.connect(f)
        cur = c.execute("select * from rocpd_kernel_dispatch limit 1")
        cols = [d[0] for d in cur.description]
        qcol = next((k for k in ("queue_id", "stream_id") if k in cols), None)
        q = (f"select s.display_name, d.start, d.end, {'d.' + qcol if qcol else '0'} "
             "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
        rows += [{"name": r[0], "start": r[1], "end": r[2], "q": r[3]} for r in c.execute(q)]
    rows.sort(key=lambda r: r["start"])
    return rows


def short(n, w):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n[:w]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--names", type=int, default=56)
    p.add_argument("--last", type=int, default=0)
    a = p.parse_args()
    rows = load(a.path)
    mb = [i for i, r in enumerate(rows) if "make_batch" in r["name"]]
    if len(mb) < 2:  # the batch is built inside conv0's forward: that kernel heads the step
        mb = [i for i, r in enumerate(rows) if "conv0_fwd_kernel<true>" in r["name"]]
    if len(mb) < 2:
        print("need two make_batch dispatches")
        return
    if a.last:
        print(f"# last {a.last} steps: span / main-queue busy / main-queue idle between its dispatches (us)")
        tot = [0.0, 0.0, 0.0]
        sel = list(zip(mb, mb[1:]))[-a.last:]
        for i0, i1 in sel:
            st = rows[i0:i1]
            mq = [r for r in st if r["q"] == st[0]["q"]]
            span = (rows[i1]["start"] - st[0]["start"]) / 1e3
            busy = sum(r["end"] - r["start"] for r in mq) / 1e3
            idle = sum(max(0, b["start"] - e["end"]) for e, b in zip(mq, mq[1:])) / 1e3
            idle += max(0, rows[i1]["start"] - mq[-1]["end"]) / 1e3
            tot = [tot[0] + span, tot[1] + busy, tot[2] + idle]
            print(f"  {span:8.1f} {busy:8.1f} {idle:8.1f}")
        n = len(sel)
        print(f"# mean  {tot[0] / n:8.1f} {tot[1] / n:8.1f} {tot[2] / n:8.1f}\n")
    step = rows[mb[-2]:mb[-1]]
    if a.last:  # the detail: the step of the window whose main queue idled least
        i0, i1 = min(list(zip(mb, mb[1:]))[-a.last:], key=lambda p: (rows[p[1]]["start"] - rows[p[0]]["start"]) - sum(
            r["end"] - r["start"] for r in rows[p[0]:p[1]] if r["q"] == rows[p[0]]["q"]))
        step = rows[i0:i1]
        mb = [i0, i1]
    t0 = step[0]["start"]
    span = (rows[mb[-1]]["start"] - t0) / 1e3
    byq = collections.defaultdict(list)
    for r in step:
        byq[r["q"]].append(r)
    main_q = step[0]["q"]
    print(f"# one step: {len(step)} dispatches, span {span:.1f} us (step head to step head), queues {len(byq)}")
    for qid, rs in sorted(byq.items(), key=lambda kv: (kv[0] != main_q, kv[0])):
        busy = sum(r["end"] - r["start"] for r in rs) / 1e3
        print(f"\n## queue {qid}{' (main)' if qid == main_q else ''}: {len(rs)} dispatches, busy {busy:.1f} us")
        prev = None
        gaps = 0.0
        for r in rs:
            gap = (r["start"] - prev) / 1e3 if prev is not None else 0.0
            gaps += max(gap, 0.0)
            print(f"{(r['start'] - t0) / 1e3:8.1f} {(r['end'] - r['start']) / 1e3:7.2f} {gap:7.2f}  "
                  f"{short(r['name'], a.names)}")
            prev = r["end"]
        print(f"# queue {qid}: idle between its dispatches {gaps:.1f} us")
    # kernel-name classes on the main queue
    cls = collections.OrderedDict((k, 0.0) for k in ("conv_gemm", "conv_xp", "splitk", "bn_", "link_", "sgd",
                                                       "head_", "make_batch", "conv0", "other"))
    for r in byq[main_q]:
        d = (r["end"] - r["start"]) / 1e3
        k = next((k for k in cls if k != "other" and k in r["name"]), "other")
        cls[k] += d
    print("\n# main-queue busy by class (us): " + ", ".join(f"{k} {v:.1f}" for k, v in cls.items() if v > 0))


if __name__ == "__main__":
    main()
