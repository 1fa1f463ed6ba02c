#!/usr/bin/env python3
"""Concurrency inside one training step of a rocprofv3 kernel trace with the
weight-gradient side stream ON: wall span, time with no kernel running on any
queue (idle), time with exactly one queue busy, per-queue busy time, and the
largest all-idle gaps.  usage: step_overlap.py <kernel_trace.csv> [top]"""
import sys

from step_timeline import step_rows


def main():
    rows = step_rows(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    ev = []
    per_q = {}
    for r in rows:
        s, e, q = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?")
        ev.append((s, 1, q))
        ev.append((e, -1, q))
        per_q[q] = per_q.get(q, 0) + (e - s)
    ev.sort()
    t0, t1 = ev[0][0], ev[-1][0]
    active = {}
    last = t0
    idle = one = many = 0
    gaps = []
    for t, d, q in ev:
        n = sum(1 for v in active.values() if v > 0)
        dt = t - last
        if n == 0 and dt > 0:
            idle += dt
            gaps.append((dt, t))
        elif n == 1:
            one += dt
        elif n > 1:
            many += dt
        active[q] = active.get(q, 0) + d
        last = t
    span = t1 - t0
    print("step span %.3f ms: idle %.3f ms, one queue busy %.3f ms, >= 2 queues %.3f ms"
          % (span / 1e6, idle / 1e6, one / 1e6, many / 1e6))
    for q, b in sorted(per_q.items(), key=lambda kv: -kv[1]):
        print("  queue %s busy %.3f ms (%.0f%% of span)" % (q, b / 1e6, 100.0 * b / span))
    for g, t in sorted(gaps, reverse=True)[:top]:
        print("  idle %7.1f us ending at +%.3f ms" % (g / 1e3, (t - t0) / 1e6))


if __name__ == "__main__":
    main()
