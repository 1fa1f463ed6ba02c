#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --kernel-trace sqlite results
(run_results.db), per training step: the steps are the intervals between
consecutive dispatches of a once-per-step marker kernel (default: the
synthetic-image kernel that starts every step), the last ``--steps`` full
intervals are averaged.  Two runs print side by side.

  python scripts/prof_db.py A.db [B.db] [--steps 8] [--top 40] [--match s1_k]"""
import argparse
import collections
import re
import sqlite3


def short(name):
    s = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", s)


def load(path, marker, steps):
    con = sqlite3.connect(path)
    rows = con.execute("select name, duration, start, end, stream_id from kernels "
                       "order by start").fetchall()
    marks = [r[2] for r in rows if marker in r[0]]
    if len(marks) < steps + 1:
        raise SystemExit("%s: only %d marker dispatches" % (path, len(marks)))
    lo, hi = marks[-steps - 1], marks[-1]
    per = collections.defaultdict(float)
    cnt = collections.Counter()
    stream = collections.defaultdict(float)
    for name, dur, st, en, sid in rows:
        if lo <= st < hi:
            k = short(name)
            per[k] += dur / 1e3 / steps
            cnt[k] += 1
            stream[sid] += dur / 1e3 / steps
    return per, cnt, stream, (hi - lo) / 1e3 / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default="")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--marker", default="synthetic_images")
    a = ap.parse_args()
    runs = [load(p, a.marker, a.steps) for p in a.dbs]
    for p, (per, cnt, stream, step) in zip(a.dbs, runs):
        print("%s: step %.1f us; kernel time per stream: %s" % (
            p, step, ", ".join("%s %.1f" % kv for kv in sorted(stream.items()))))
    keys = set().union(*[r[0].keys() for r in runs])
    keys = sorted((k for k in keys if a.match in k), key=lambda k: -runs[0][0].get(k, 0.0))
    for k in keys[:a.top]:
        cols = ["%8.1f %4d" % (r[0].get(k, 0.0), r[1][k] // a.steps) for r in runs]
        print(" | ".join(cols), k[:100])


if __name__ == "__main__":
    main()
