#!/usr/bin/env python3
"""Per-kernel HBM traffic and achieved bandwidth over the last training step
of a scripts/pmc_bytes.sh run (FETCH_SIZE / WRITE_SIZE counter passes, KB).

usage: bytes_roofline.py <outdir>"""
import collections
import csv
import glob
import os
import sys


def load(outdir, counter, marker="opt_step_k"):
    tr = glob.glob(os.path.join(outdir, counter, "**", "*kernel_trace.csv"), recursive=True)[0]
    cc = glob.glob(os.path.join(outdir, counter, "**", "*counter_collection.csv"),
                   recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    step = rows[ends[-2] + 1:ends[-1] + 1]
    val = collections.defaultdict(float)
    for r in csv.DictReader(open(cc)):
        val[r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = []
    for r in step:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out.append((r["Kernel_Name"].split("(")[0][:64], us, val.get(r["Dispatch_Id"], 0.0) * 1024))
    return out


def main():
    d = sys.argv[1]
    f = load(d, "FETCH_SIZE")
    w = load(d, "WRITE_SIZE")
    assert len(f) == len(w), (len(f), len(w))
    agg = collections.OrderedDict()
    tot_t = tot_b = 0.0
    for (name, us, rb), (_, us2, wb) in zip(f, w):
        t = min(us, us2)
        a = agg.setdefault(name, [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += t
        a[2] += rb
        a[3] += wb
        tot_t += t
        tot_b += rb + wb
    print("one step: %.2f ms kernel time, %.2f GB HBM traffic -> %.2f TB/s average; "
          "at 5.4 TB/s the traffic alone needs %.2f ms"
          % (tot_t / 1e3, tot_b / 1e9, tot_b / tot_t / 1e6, tot_b / 5.4e12 * 1e3))
    print("%-64s %5s %9s %9s %9s %7s" % ("kernel", "calls", "ms", "read GB", "write GB", "TB/s"))
    for name, (c, t, rb, wb) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-64s %5d %9.3f %9.3f %9.3f %7.2f" % (name, c, t / 1e3, rb / 1e9, wb / 1e9,
                                                     (rb + wb) / t / 1e6 if t else 0))


if __name__ == "__main__":
    main()
