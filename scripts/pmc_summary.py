#!/usr/bin/env python3
"""Summarize a rocprofv3 --pmc counter CSV per (kernel, grid size).

usage: pmc_summary.py <run_counter_collection.csv> [--filter substr]
Prints, per kernel/grid group, the mean of every collected counter and the
SQ wait breakdown (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY over
WAVE_CYCLES) when those counters are present.
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else None
    groups = collections.OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if flt and flt not in name:
                continue
            grid = row.get("Grid_Size", row.get("Grid_Size_X", ""))
            key = (name[:60], grid)
            g = groups.setdefault(key, collections.defaultdict(list))
            g[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for (name, grid), ctr in groups.items():
        mean = {k: sum(v) / len(v) for k, v in ctr.items()}
        print("%s grid=%s" % (name, grid))
        for k in sorted(mean):
            print("    %-28s %14.0f" % (k, mean[k]))
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            parts = ["%s %.1f%%" % (k.replace("SQ_", ""), 100 * mean[k] / wc)
                     for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                     if k in mean]
            print("    -> " + ", ".join(parts))


if __name__ == "__main__":
    main()
