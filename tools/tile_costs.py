#!/usr/bin/env python3
"""Per-tile phase costs of a profile run (tools/profile_phases.py RAW=...,
QHUFF_PROFILE build; iteration it + 8, slot 5 holds the tile id of
iteration it) joined with the tile's shape, for the corpus workload:
which tiles are slow in the codec, and which in the slow path (gather
phase, where big tiles run).

usage: python tools/tile_costs.py raw.npz [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from qhuff import workload as W
    import oracle_lib as O
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    d, o = W.corpus_batch(n, os.path.join(ROOT, "tests", "golden", "data"))
    h, ho = O.encode_batch(d, o, 0)
    o = o.astype(np.int64)
    ho = ho.astype(np.int64)
    nt = (n + 63) // 64
    t0 = np.arange(nt) * 64
    t1 = np.minimum(t0 + 64, n)
    hl = np.diff(ho)
    rl = np.diff(o)
    span = ho[t1] - ho[t0]
    mx = np.maximum.reduceat(hl, t0)
    ncoop = np.add.reduceat((hl > 128).astype(np.int64), t0)
    lens = W.RFC_LEN[d]
    nlong = np.add.reduceat(np.concatenate([[0], (lens > 13).astype(np.int64)])[
        np.concatenate([[0], np.cumsum(rl)])[t0]:][:0], [0]) if False else None
    plong = np.concatenate([[0], np.cumsum(lens > 13)])
    nlong = plong[o[t1]] - plong[o[t0]]
    outsz = o[t1] - o[t0]
    R = np.load(sys.argv[1])
    for tag in ("decode", "encode"):
        p = R[tag].reshape(-1, 16, 12).astype(np.int64)
        live = p[:, :8, 0] != 0
        rows, its = np.nonzero(live[:, :7])
        tid = p[rows, its + 8, 5]
        codec = p[rows, its, 3] - p[rows, its, 2]
        flush = p[rows, its, 5] - p[rows, its, 4]
        gath = p[rows, its, 6] - p[rows, its, 5]
        ok = (tid < nt) & (p[rows, its, 6] != 0)
        tid, codec, flush, gath = tid[ok], codec[ok], flush[ok], gath[ok]
        big = (span[tid] > 3072 - 32) | (outsz[tid] > 3000)
        print("%s: %d tiles seen" % (tag, len(tid)))
        for name, v in (("codec", codec), ("gather(+slow path)", gath)):
            print("  %-20s p50 %8.0f p90 %8.0f p99 %8.0f max %9.0f cycles"
                  % (name, np.median(v), np.percentile(v, 90),
                     np.percentile(v, 99), v.max()))
        print("  big tiles %d: gather p50 %.0f max %.0f" % (
            big.sum(), np.median(gath[big]) if big.any() else 0,
            gath[big].max() if big.any() else 0))
        q = p[:, 15, :4]
        okb = (q[:, 0] != 0) & (q[:, 3] != 0)
        if okb.any():
            a1 = q[okb, 1] - q[okb, 0]
            a2 = q[okb, 2] - q[okb, 1]
            a3 = q[okb, 3] - q[okb, 2]
            print("  big tiles (last per wave, %d): sizes pass p50 %.0f max %.0f"
                  " | base wait p50 %.0f max %.0f | output pass p50 %.0f max %.0f"
                  % (okb.sum(), np.median(a1), a1.max(), np.median(a2), a2.max(),
                     np.median(a3), a3.max()))
        if tag == "decode":
            q = p[:, 15, :]
            okc = (q[:, 4] != 0) & (q[:, 8] != 0)
            if okc.any():
                A = q[okc, 5] - q[okc, 4]
                B = q[okc, 6] - q[okc, 5]
                Cn = q[okc, 7] - q[okc, 6]
                Wt = q[okc, 8] - q[okc, 7]
                rd = q[okc, 9]
                print("  coop (last per wave, %d): A p50 %.0f p90 %.0f | B p50 %.0f"
                      " p90 %.0f (rounds p50 %.0f max %d) | count p50 %.0f | W p50 %.0f"
                      " p90 %.0f" % (okc.sum(), np.median(A), np.percentile(A, 90),
                                     np.median(B), np.percentile(B, 90),
                                     np.median(rd), rd.max(), np.median(Cn),
                                     np.median(Wt), np.percentile(Wt, 90)))
        top = np.argsort(-codec)[:12]
        print("  slowest codecs: cycles | span maxhl ncoop nlong")
        for k in top:
            t = tid[k]
            print("   %8d | %5d %5d %3d %4d" % (codec[k], span[t], mx[t],
                                               ncoop[t], nlong[t]))
        # codec cost vs shape (mean cycles)
        for lab, m in (("no coop, no long", (ncoop[tid] == 0) & (nlong[tid] == 0)),
                       ("coop", ncoop[tid] > 0), ("long codes", nlong[tid] > 0)):
            if m.any():
                print("  codec %-18s %6d tiles mean %8.0f p90 %8.0f"
                      % (lab, m.sum(), codec[m].mean(), np.percentile(codec[m], 90)))


if __name__ == "__main__":
    main()
