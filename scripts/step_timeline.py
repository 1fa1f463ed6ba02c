#!/usr/bin/env python3
"""Per-dispatch timeline of one training step from a rocprofv3 kernel trace
(the last complete step: dispatches after the second-to-last optimizer
kernel).  usage: step_timeline.py <kernel_trace.csv> [--min-us X]"""
import argparse
import csv


def step_rows(path, marker="opt_step_k", back=1):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    return rows[ends[-1 - back] + 1:ends[-back] + 1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    for i, r in enumerate(step_rows(a.path)):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if us < a.min_us:
            continue
        name = r["Kernel_Name"].split("(")[0]
        print("%4d %-58s wg %7d x %3s vgpr %3s lds %6s %8.1f" % (
            i, name[:58], int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1),
            r["Workgroup_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"], us))


if __name__ == "__main__":
    main()
