#!/usr/bin/env python3
"""Cross-wave analysis of a phase-profile dump (tools/profile_phases.py
RAW=..., QHUFF_PROFILE build).  Stamps of different XCDs come from
different s_memtime counters, so every wave's stamps are placed on the
wall clock through its own s_memrealtime stamp (slot 11 of iteration 0,
100 MHz) at the shader clock.

  * look-back of the flushes that resolve iteration-k tiles, against the
    moment the last tile before each one published its aggregate (slot 9,
    tile ids in slot 5 of iteration it + 8);
  * tile time by XCD, by wave of the workgroup and by age rank on its SIMD;
  * the slowest waves, phase by phase;
  * the drain (iteration 14 slots 6/7/8) when the build stamps it.

usage: python tools/wave_report.py raw.npz [n_tiles]"""
import sys

import numpy as np

ITERS, SLOTS, W = 16, 12, 12


def report(tag, p, ntile):
    p = p.reshape(-1, ITERS, SLOTS).astype(np.int64)
    p = p[p[:, 0, 0] != 0]
    nw = len(p)
    rt0 = p[:, 0, 11] * 10.0                       # ns
    mt0 = p[:, 0, 0]
    nit = (p[:, :8, 0] != 0).sum(1)
    last = nit - 1
    dt = (p[np.arange(nw), last, 11] - p[:, 0, 11]) * 10.0
    ghz = np.median(((p[np.arange(nw), last, 0] - mt0) / dt)[dt > 0])
    base = rt0.min()

    def g(it, sl):
        return rt0 + (p[:, it, sl] - mt0) / ghz - base

    print("%s: %d waves, shader clock %.3f GHz" % (tag, nw, ghz))
    tid = p[:, 8:15, 5]
    pub = np.full(ntile, np.nan)
    for it in range(7):
        ok = (p[:, it, 9] != 0) & (tid[:, it] < ntile) & (p[:, it, 0] != 0)
        pub[tid[ok, it]] = g(it, 9)[ok]
    if np.isfinite(pub).sum() > ntile // 2:
        cm = np.fmax.accumulate(np.nan_to_num(pub, nan=0.0))
        for it in (3, 4, 5):
            ok = (p[:, it, 7] != 0) & (p[:, it, 4] != 0)
            if not ok.any():
                continue
            t = tid[ok, it - 3]
            need = np.where(t > 0, cm[np.maximum(t - 1, 0)], 0.0)
            fs, lb = g(it, 4)[ok], g(it, 7)[ok]
            late = need - fs
            print("  flush of iteration %d (iteration-%d tiles): look-back p50 %.0f"
                  " p90 %.0f ns; last predecessor's aggregate - flush start p50 %.0f"
                  " p90 %.0f ns" % (it, it - 3, np.median(lb - fs),
                                    np.percentile(lb - fs, 90), np.median(late),
                                    np.percentile(late, 90)))
    rows = np.nonzero(nit >= 5)[0]
    per = (p[rows, 4, 11] - p[rows, 0, 11]) * 10.0 / 4
    blk, w = rows // W, rows % W
    for name, key, n in (("XCD", blk % 8, 8), ("wave", w, W), ("age rank", w >> 2, 3)):
        print("  ns per tile (first 4) by %-8s %s" % (
            name, " ".join("%5.0f" % per[key == k].mean() for k in range(n))))
    end = np.array([g(nit[i] - 1, 6)[i] for i in range(nw)])
    print("  wave end (ns): p50 %.0f p90 %.0f p99 %.0f max %.0f" % tuple(
        np.percentile(end, [50, 90, 99, 100])))
    for i in np.argsort(-end)[:6]:
        ph = ["[%s]" % ",".join("%d" % ((p[i, it, k + 1] - p[i, it, k]) / 100)
                                 for k in range(6)) for it in range(nit[i])]
        print("   w%4d blk %3d wave %2d tiles %d end %.0f  %s" % (
            i, i // W, i % W, nit[i], end[i], " ".join(ph)))
    d0, d1 = p[:, 14, 6], p[:, 14, 7]
    ok = (d0 != 0) & (d1 != 0)
    if ok.any():
        dur = (d1 - d0)[ok]
        de = (p[ok, 14, 8] * 10.0 - base)
        print("  drain: cycles p50 %d p90 %d max %d | ends (ns) p50 %.0f p99 %.0f"
              " max %.0f" % (np.median(dur), np.percentile(dur, 90), dur.max(),
                             np.median(de), np.percentile(de, 99), de.max()))


def main():
    z = np.load(sys.argv[1])
    ntile = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    for tag in ("encode", "decode"):
        report(tag, z[tag], ntile)


if __name__ == "__main__":
    main()
