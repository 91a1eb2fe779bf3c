#!/usr/bin/env python3
"""Where a 1M-string launch's end goes, from the raw phase stamps of a
QHUFF_PROFILE build (tools/profile_phases.py with RAW=path.npz).

Per kernel: the spread of iteration ends (cycles relative to each wave's own
first stamp), the distance from the last round's median end to the kernel's
last end, the first-flush wait (iteration kDepth's
flush against the steady state, item 3), and which waves end last: their
tile count, age rank on the SIMD (wave >> 2 in the workgroup) and where
their last iteration's time went.

usage: python tools/tail_report.py raw.npz [depth]"""
import sys

import numpy as np

ITERS, SLOTS, W = 16, 12, 12
NAMES = ["top wait", "stage+loads+polls", "codec+scan", "start+emit+wait",
         "flush", "gather"]


def report(tag, p, depth):
    p = p.reshape(-1, ITERS, SLOTS).astype(np.int64)
    live = p[:, :, 0] != 0
    rows = np.nonzero(live[:, 0])[0]
    nit = live[rows].sum(axis=1)
    t0 = p[rows, 0, 0]
    last = nit - 1
    end = p[rows, last, 6] - t0                      # own clock, cycles
    # wall clock (100 MHz) of each wave's end, relative to the earliest start
    r0 = p[rows, 0, 11]
    base = r0.min()
    end_us = (p[rows, last, 11] - base) * 0.01 + (p[rows, last, 6]
                                                  - p[rows, last, 0]) / 2200.0
    print("%s: %d waves, %.2f tiles/wave" % (tag, len(rows), nit.mean()))
    full = nit == nit.max()
    lr = nit.max() - 1
    lr_end = p[rows[full], lr, 6] - t0[full]
    print("  last round (iteration %d, %d waves): end p50 %.0f max %.0f cycles;"
          " all waves' end p50 %.0f max %.0f; kernel end - last-round p50 %.0f"
          % (lr, full.sum(), np.median(lr_end), lr_end.max(), np.median(end),
             end.max(), end.max() - np.median(lr_end)))
    print("  wave end wall clock: p50 %.2f p90 %.2f p99 %.2f max %.2f us"
          % tuple(np.percentile(end_us, [50, 90, 99, 100])))
    # first flush (iteration depth) vs the iterations after it
    fl = p[rows, :, 5] - p[rows, :, 4]
    ok = live[rows] & (p[rows, :, 5] != 0) & (p[rows, :, 4] != 0)
    per_it = [np.median(fl[:, i][ok[:, i]]) if ok[:, i].any() else 0
              for i in range(ITERS)]
    later = [x for x in per_it[depth + 1:] if x]
    print("  flush p50 by iteration: %s  (first flush %.0f vs later %.0f)"
          % (" ".join("%.0f" % x for x in per_it[:nit.max()]), per_it[depth],
             np.median(later) if later else 0))
    # the last 1% of waves to end
    k = max(1, len(rows) // 100)
    idx = np.argsort(-end_us)[:k]
    wv = rows[idx] % W
    print("  last %d waves: tiles %s | age rank %s | XCD %s"
          % (k, np.bincount(nit[idx], minlength=7)[4:].tolist(),
             np.bincount(wv >> 2, minlength=3).tolist(),
             np.bincount((rows[idx] // W) % 8, minlength=8).tolist()))
    li = last[idx]
    ph = [(p[rows[idx], li, j + 1] - p[rows[idx], li, j]).mean()
          for j in range(6)]
    print("  their last iteration: " + ", ".join(
        "%s %.0f" % (n, x) for n, x in zip(NAMES, ph)))


def main():
    d = np.load(sys.argv[1])
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for tag in ("encode", "decode"):
        if tag in d:
            report(tag, d[tag], depth)


if __name__ == "__main__":
    main()
