#!/usr/bin/env python3
"""Collects the JSON lines of a zoo run (gpurun_out/<tag>/*.log) into
profiles/<dest>/<model>_<batch>.json and prints a markdown table
(img/s, ms/step, host ms/step, launch tape, tape host time).

  python scripts/zoo_table.py gpurun_out/zoo_r9a [gpurun_out/zoo_r9b ...] --dest profiles/zoo_r9"""
import argparse
import glob
import json
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--dest", default=None)
    a = ap.parse_args()
    rows = []
    for d in a.dirs:
        for path in sorted(glob.glob(os.path.join(d, "*.log"))):
            text = open(path, errors="replace").read()
            js = [l for l in text.splitlines() if l.startswith('{"metric"')]
            if not js:
                continue
            r = json.loads(js[-1])
            m = re.search(r"tape host time per replayed step: ([0-9.]+) ms over (\d+) calls \((\d+) raw",
                          text)
            r["tape_host"] = (float(m.group(1)), int(m.group(2)), int(m.group(3))) if m else None
            name = os.path.basename(path)[:-4]
            rows.append((name, r))
            if a.dest:
                os.makedirs(a.dest, exist_ok=True)
                with open(os.path.join(a.dest, name + ".json"), "w") as f:
                    f.write(js[-1] + "\n")
    print("| model_batch | img/s | ms/step | host ms/step | tape | tape host ms (calls, raw) |")
    print("|---|---|---|---|---|---|")
    for name, r in rows:
        th = r["tape_host"]
        print("| %s | %.0f | %.2f | %.2f | %s | %s |" % (
            name, r["value"], r["ms_per_step"], r.get("host_ms_per_step") or 0,
            r["config"].get("launch_tape"),
            "%.2f (%d, %d)" % th if th else "-"))


if __name__ == "__main__":
    main()
