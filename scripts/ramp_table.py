#!/usr/bin/env python3
"""Attribute the start-up step-time ramp to kernels: from one rocprofv3 kernel trace (.db) of a
long native-engine run (scripts/ramp_run.py), split the dispatches into steps at each step-head
kernel (conv0_fwd / make_batch on the main queue) and compare two step windows (default 5-25 vs
200-220): per kernel name and queue, mean duration per step early vs late, the step span (head to
head) and the main queue's idle time — which named kernels carry the span delta.

    python3 scripts/ramp_table.py gpurun_out/ramp [--early 5:25] [--late 200:220]
"""
import argparse
import collections
import glob
import os
import sqlite3

HEADS = ("conv0_fwd_kernel", "make_batch_kernel")


def load(path):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*.db"), recursive=True):
        c = sqlite3.connect(f)
        cols = [d[0] for d in c.execute("select * from rocpd_kernel_dispatch limit 1").description]
        qcol = next((k for k in ("queue_id", "stream_id") if k in cols), None)
        q = (f"select s.display_name, d.start, d.end, {'d.' + qcol if qcol else '0'} from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
        rows += [(r[0], r[1], r[2], r[3]) for r in c.execute(q)]
    rows.sort(key=lambda r: r[1])
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("path")
    p.add_argument("--early", default="5:25")
    p.add_argument("--late", default="200:220")
    a = p.parse_args()
    rows = load(a.path)
    heads = [r for r in rows if any(h in r[0] for h in HEADS)]
    main_q = collections.Counter(r[3] for r in heads).most_common(1)[0][0]
    heads = [r for r in heads if r[3] == main_q]
    starts = [r[1] for r in heads]
    steps = collections.defaultdict(list)  # step index -> dispatches started in [head_k, head_k+1)
    j = 0
    for r in rows:
        while j + 1 < len(starts) and r[1] >= starts[j + 1]:
            j += 1
        if r[1] >= starts[0]:
            steps[j].append(r)

    def window(spec):
        lo, hi = (int(x) for x in spec.split(":"))
        return [k for k in range(lo, hi) if k + 1 < len(starts)]

    def stats(ks):
        per = collections.defaultdict(float)
        span = idle = 0.0
        for k in ks:
            span += (starts[k + 1] - starts[k]) / 1e3
            mq = sorted((r for r in steps[k] if r[3] == main_q), key=lambda r: r[1])
            busy = sum((r[2] - r[1]) / 1e3 for r in mq)
            idle += (starts[k + 1] - starts[k]) / 1e3 - busy
            for r in steps[k]:
                per[(short(r[0]), "main" if r[3] == main_q else f"q{r[3]}")] += (r[2] - r[1]) / 1e3
        n = max(len(ks), 1)
        return {k: v / n for k, v in per.items()}, span / n, idle / n

    ke, kl = window(a.early), window(a.late)
    pe, se, ie = stats(ke)
    pl, sl, il = stats(kl)
    ds = se - sl
    print(f"# steps in trace: {len(starts) - 1}; early {a.early} ({len(ke)} steps) vs late {a.late} ({len(kl)} steps)")
    print(f"# step span (head to head): early {se:.1f} us, late {sl:.1f} us, delta {ds:+.1f} us")
    print(f"# main-queue idle per step: early {ie:.1f} us, late {il:.1f} us, delta {ie - il:+.1f} us")
    keys = sorted(set(pe) | set(pl), key=lambda k: -(pe.get(k, 0) - pl.get(k, 0)))
    main_delta = sum(pe.get(k, 0) - pl.get(k, 0) for k in keys if k[1] == "main")
    print(f"# main-queue kernel time delta {main_delta:+.1f} us = {100 * main_delta / ds if ds else 0:.0f} % of the span "
          f"delta; idle {100 * (ie - il) / ds if ds else 0:.0f} %")
    print(f"{'kernel':70s} {'queue':>5s} {'early_us':>9s} {'late_us':>9s} {'delta':>8s} {'%span':>6s} {'ratio':>6s}")
    for k in keys:
        e, l = pe.get(k, 0.0), pl.get(k, 0.0)
        if abs(e - l) < 0.05 and e < 1.0:
            continue
        print(f"{k[0]:70s} {k[1]:>5s} {e:9.2f} {l:9.2f} {e - l:+8.2f} {100 * (e - l) / ds if ds else 0:6.1f} "
              f"{e / l if l else 0:6.3f}")


if __name__ == "__main__":
    main()
