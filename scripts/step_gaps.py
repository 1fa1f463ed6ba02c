#!/usr/bin/env python3
"""Idle gaps inside one training step of a rocprofv3 kernel trace (every
kernel on one stream, KFB_WGRAD_STREAM=0): total idle time and the largest
gaps with the kernels on either side.  usage: step_gaps.py <kernel_trace.csv>"""
import csv
import sys

from step_timeline import step_rows


def main():
    rows = step_rows(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    gaps = []
    t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
    busy = 0
    end = None
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and s > end:
            gaps.append((s - end, i))
        busy += e - max(s, end or s)
        end = max(end or e, e)
    idle = sum(g for g, _ in gaps)
    print("step span %.3f ms, kernels %d, idle %.3f ms in %d gaps" % (
        (t1 - t0) / 1e6, len(rows), idle / 1e6, len(gaps)))
    name = lambda r: r["Kernel_Name"].split("(")[0][:48]
    for g, i in sorted(gaps, reverse=True)[:top]:
        print("%8.1f us  after %4d %-48s before %s" % (g / 1e3, i - 1, name(rows[i - 1]),
                                                       name(rows[i])))


if __name__ == "__main__":
    main()
