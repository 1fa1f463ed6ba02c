#!/usr/bin/env python3
"""Per-layer speed-of-light table of the ResNet-50 convolutions from an
autotune log (``KFB_AUTOTUNE_LOG=1 python bench.py ...``): every geometry's
candidates were timed in the network's first step on the real operands with
the real fused epilogue (BN statistics in the forward, the producer BN's
backward epilogue in the data gradient, the slab fold in the weight
gradient), so the chosen kernel's time is the in-network cost of the layer
with the chip to itself.

For each layer: pass, chosen kernel, us, calls per step (ResNet-50 v1),
TF/s, % of the practical MFMA peak (1.55 PF/s, profiles/r8_mfma_forms.txt)
and % of the byte bound (operand + output bytes at 6 TB/s), then the totals
per pass and the time a layer would take at the better of the two bounds.

  python scripts/sol_table.py gpurun_out/<tag>/tune.log
"""
import re
import sys
from collections import defaultdict

PEAK = 1.55e15   # bf16 MFMA, measured practical peak (random operands, every CU)
BW = 6.0e12      # HBM bytes/s a streaming kernel reaches (6.0-6.3 measured)

# (H, Cin, Cout, k, stride) -> calls per step in ResNet-50 v1 (scripts/bench_conv.py)
COUNT = {
    (224, 3, 64, 7, 2): 1, (56, 64, 256, 1, 1): 4, (56, 64, 64, 1, 1): 1,
    (56, 256, 64, 1, 1): 2, (56, 64, 64, 3, 1): 3, (56, 256, 512, 1, 2): 1,
    (56, 256, 128, 1, 2): 1, (28, 128, 128, 3, 1): 4, (28, 128, 512, 1, 1): 4,
    (28, 512, 128, 1, 1): 3, (28, 512, 1024, 1, 2): 1, (28, 512, 256, 1, 2): 1,
    (14, 256, 256, 3, 1): 6, (14, 256, 1024, 1, 1): 6, (14, 1024, 256, 1, 1): 5,
    (14, 1024, 2048, 1, 2): 1, (14, 1024, 512, 1, 2): 1, (7, 512, 512, 3, 1): 3,
    (7, 512, 2048, 1, 1): 3, (7, 2048, 512, 1, 1): 2,
}


def parse(path):
    rows = []
    for line in open(path):
        m = re.match(r"\[autotune\] (igemm|wgrad) \((.*?)\)( \+bn)?: (.*)", line.strip())
        if not m:
            continue
        geo = tuple(int(v) for v in m.group(2).split(","))
        best, t = m.group(4).split("  ")[0].rsplit(" ", 1)
        rows.append((m.group(1), geo, bool(m.group(3)), best, float(t)))
    return rows


def layer(kind, geo, bn):
    """(H, Cin, Cout, k, stride, pass) of a logged geometry, or None."""
    if kind == "wgrad":
        n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, cout = geo
        if C == 8:
            return (224, 3, 64, 7, 2, "wgrad")
        return (H, C, cout, KH, sh, "wgrad")
    n, H, W, C, OH, OW, KH, KW, sh, sw, pt, pl, ncol, YH, YW, ys = geo[:16]
    if C == 8:
        return (224, 3, 64, 7, 2, "fwd")
    if ys == 2:  # strided 1x1 data gradient written as a scatter
        return (YH, ncol, C, 1, 2, "dgrad")
    if bn or (KH == 3 and (H, C) in ((56, 64), (28, 128), (14, 256), (7, 512))
              and (H, C, ncol, KH, 1) not in COUNT):
        # data gradient (stride 1): dY [.., Cout] -> dX [.., Cin]
        return (H, ncol, C, KH, 1, "dgrad")
    if (H, C, ncol, KH, sh) in COUNT:
        return (H, C, ncol, KH, sh, "fwd")
    if (H, ncol, C, KH, 1) in COUNT:
        return (H, ncol, C, KH, 1, "dgrad")
    return None


def main():
    rows = parse(sys.argv[1])
    seen = {}
    for kind, geo, bn, best, t in rows:
        L = layer(kind, geo, bn)
        if L is None or L in seen:
            continue
        seen[L] = (best, t)
    tot = defaultdict(float)
    sol = defaultdict(float)
    print("%-26s %6s %-12s %8s %4s %7s %6s %6s %8s" % ("layer", "pass", "kernel", "us", "n",
                                                      "TF/s", "%mfma", "%bytes", "bound_us"))
    for L in sorted(seen, key=lambda l: (-l[0], l[1], l[2], l[5])):
        H, cin, cout, k, s, pas = L
        cnt = COUNT.get((H, cin, cout, k, s), 0)
        best, t = seen[L]
        oh = H // s if k == 1 else (H + s - 1) // s if k != 7 else 112
        m = 256 * oh * oh
        flops = 2.0 * m * cout * k * k * cin
        xb = 256 * H * H * cin * 2
        if k == 1 and s == 2 and pas != "dgrad":
            xb //= 4  # a strided 1x1 reads only the sampled pixels
        yb = m * cout * 2
        byts = xb + yb + (cout * k * k * cin * 4 if pas == "wgrad" else 0)
        if pas == "dgrad" and k == 1:
            byts += xb  # producer-BN input read by the fused backward epilogue
        tf = flops / (t * 1e-6) / 1e12
        bound = max(flops / PEAK, byts / BW) * 1e6
        tot[pas] += t * cnt
        sol[pas] += bound * cnt
        print("%-26s %6s %-12s %8.1f %4d %7.0f %5.0f%% %5.0f%% %8.1f" % (
            "%dx%d %d->%d k%d s%d" % (H, H, cin, cout, k, s), pas, best[:12], t, cnt, tf,
            100 * flops / (t * 1e-6) / PEAK, 100 * byts / (t * 1e-6) / BW, bound))
    print()
    for pas in ("fwd", "dgrad", "wgrad"):
        print("%-6s %8.0f us/step in-network-isolated vs %8.0f us at the bound (%.0f%%)" % (
            pas, tot[pas], sol[pas], 100 * sol[pas] / max(tot[pas], 1e-9)))
    print("all    %8.0f us/step vs %8.0f us at the bound" % (sum(tot.values()), sum(sol.values())))


if __name__ == "__main__":
    main()
