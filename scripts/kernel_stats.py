#!/usr/bin/env python3
"""Summarize a rocprofv3 --kernel-trace run (rocpd sqlite or kernel_stats.csv)
into a per-kernel table: calls, total ms, avg us, % of GPU time.

usage: kernel_stats.py <run_results.db | kernel_trace.csv> [--steps N] [--top K]
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
    return [(r[0], (r[2] - r[1]) / 1e3) for r in rows]  # us


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    ks = from_db(a.path) if a.path.endswith(".db") else from_csv(a.path)
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
