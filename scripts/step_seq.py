#!/usr/bin/env python3
"""Every dispatch of one training step from a rocprofv3 --kernel-trace
database, in start order: stream, start / end / duration (us from the step
start), workgroups, kernel; then the idle time per stream (holes between
consecutive kernels of a stream).  The step is the interval between two
dispatches of the once-per-step marker kernel (``--which`` counts back from
the last one).

  python scripts/step_seq.py run_results.db [--which 2] [--marker synthetic_images]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--which", type=int, default=2)
    ap.add_argument("--marker", default="synthetic_images")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, duration, start, end, stream_id, grid_x, grid_y, grid_z, "
                       "workgroup_x, workgroup_y, workgroup_z from kernels order by start").fetchall()
    marks = [r[2] for r in rows if a.marker in r[0]]
    lo, hi = marks[-a.which - 1], marks[-a.which]
    last_end = {}
    holes = defaultdict(float)
    nholes = defaultdict(int)
    busy = defaultdict(float)
    for n, d, s, e, sid, gx, gy, gz, wx, wy, wz in rows:
        if not lo <= s < hi:
            continue
        n = re.sub(r"^void ", "", re.sub(r"\(.*", "", n)).replace("_ZN3kfb", "")
        wgs = (gx // max(wx, 1)) * (gy // max(wy, 1)) * (gz // max(wz, 1))
        print("%s %9.1f %9.1f %7.1f %7d %s" % (sid, (s - lo) / 1e3, (e - lo) / 1e3, d / 1e3, wgs,
                                               n[:80]))
        if sid in last_end and s - last_end[sid] > 500:
            holes[sid] += (s - last_end[sid]) / 1e3
            nholes[sid] += 1
        last_end[sid] = e
        busy[sid] += d / 1e3
    print("# step %.1f us" % ((hi - lo) / 1e3))
    for sid in sorted(busy):
        print("# stream %s: busy %.1f us, %d holes > 0.5 us totalling %.1f us"
              % (sid, busy[sid], nholes[sid], holes[sid]))


if __name__ == "__main__":
    main()
