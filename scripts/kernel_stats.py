#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace run (rocpd sqlite or kernel_stats.csv)
into a per-kernel table: calls, total ms, avg us, % of GPU time.

usage: kernel_stats.py <run_results.db | kernel_trace.csv> [--steps N] [--top K]
                       [--last-steps N [--marker opt_step_k]]

--last-steps N keeps only the dispatches of the last N training steps (a step
ends with the optimizer kernel named by --marker), which excludes warmup and
the per-geometry kernel autotune trials; it also reports the GPU-busy vs wall
time of that window (launch gaps).
"""
import argparse
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name, n=90):
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels").fetchall()
    return [(r[0], r[1], r[2]) for r in rows]  # ns


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last-steps", type=int, default=0)
    ap.add_argument("--marker", default="opt_step_k")
    a = ap.parse_args()
    raw = sorted(from_db(a.path) if a.path.endswith(".db") else from_csv(a.path),
                 key=lambda r: r[1])
    if a.last_steps:
        ends = [i for i, r in enumerate(raw) if a.marker in r[0]]
        if len(ends) > a.last_steps:
            raw = raw[ends[-a.last_steps - 1] + 1:ends[-1] + 1]
            a.steps = a.last_steps
            wall = (raw[-1][2] - raw[0][1]) / 1e6
            busy = sum(r[2] - r[1] for r in raw) / 1e6
            print("window: last %d steps, wall %.2f ms/step, GPU busy %.2f ms/step (%.1f%%)"
                  % (a.last_steps, wall / a.last_steps, busy / a.last_steps, 100 * busy / wall))
    ks = [(r[0], (r[2] - r[1]) / 1e3) for r in raw]
    agg = defaultdict(lambda: [0, 0.0])
    for name, us in ks:
        agg[name][0] += 1
        agg[name][1] += us
    total = sum(v[1] for v in agg.values())
    print("total kernel time: %.1f ms over %d dispatches" % (total / 1e3, len(ks)))
    if a.steps:
        print("per step: %.2f ms" % (total / 1e3 / a.steps))
    print("%-92s %7s %10s %9s %6s" % ("kernel", "calls", "total_ms", "avg_us", "%"))
    for name, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print("%-92s %7d %10.2f %9.1f %6.2f" % (short(name), c, us / 1e3, us / c, 100 * us / total))


if __name__ == "__main__":
    main()
