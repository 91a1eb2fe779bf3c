#!/usr/bin/env python3
"""Per-phase timing of the persistent tile kernels from QHUFF_TRACE stamps.

  python tools/trace_report.py            # run enc+dec of N strings, report
Slots per tile (see qhuff_device.h stamp()):
  0 realtime at iteration start (wave 0)   1 memtime, iteration start
  2 wave 0 codec done                      3 store wave codec done
  4 wave 0 past barrier 1                  5 store wave: finish starts
  6 store wave: finish + publish done      7 wave 0 past the last barrier
  11-13 (in the finished tile's own record) look-back start, look-back
  done, copy-out done; 14 look-back re-polls; 15 workgroup
Diagnostic only: tracing synchronises after every launch."""
import os
import struct
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np


def read(path):
    recs = []
    with open(path, "rb") as f:
        b = f.read()
    p = 0
    while p + 20 <= len(b):
        magic, kind, tiles, grid, slots = struct.unpack_from("<5I", b, p)
        assert magic == 0x32525451
        p += 20
        st = np.frombuffer(b, dtype=np.uint64, count=slots * tiles, offset=p)
        p += 8 * slots * tiles
        recs.append((kind, tiles, grid, st.reshape(tiles, slots).astype(np.int64)))
    return recs


def report(kind, tiles, grid, s):
    name = "enc" if kind == 0 else "dec"
    rt = s[:, 0]
    span_us = (rt.max() - rt.min()) / 100.0
    # consecutive iterations of one workgroup (slot 15 = workgroup)
    order = np.lexsort((rt, s[:, 15]))
    wg = s[order, 15]
    same = wg[1:] == wg[:-1]
    t = order[:-1][same]
    nx = order[1:][same]
    dmt = s[nx, 1] - s[t, 1]
    drt = s[nx, 0] - s[t, 0]
    clk = np.median(dmt / np.maximum(drt, 1)) * 100e6
    cyc = lambda x: x / clk * 1e6                     # cycles -> us
    ph = {
        "codec wave0": s[:, 2] - s[:, 1],
        "codec store wave": s[:, 3] - s[:, 1],
        "barrier1 wait (w0)": s[:, 4] - s[:, 2],
        "finish+publish (store)": s[:, 6] - s[:, 5],
        "store wave idle before finish": s[:, 5] - s[:, 3],
        "w0 after barrier1 -> end": s[:, 7] - s[:, 4],
        "look-back (own record)": s[:, 12] - s[:, 11],
        "copy-out+offsets (own record)": s[:, 13] - s[:, 12],
    }
    print("%s: tiles %d grid %d  first-start..last-start %.1f us  clock %.2f GHz"
          % (name, tiles, grid, span_us, clk / 1e9))
    first = np.array([rt[s[:, 15] == w].min() for w in np.unique(s[:, 15])])
    print("   launch ramp (first-iteration start spread): %.2f us"
          % ((first.max() - first.min()) / 100.0))
    for k, v in ph.items():
        if len(v) == 0:
            continue
        v = cyc(v.astype(np.float64))
        print("   %-32s mean %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us"
              % (k, v.mean(), np.median(v), np.percentile(v, 90), v.max()))
    it = cyc(dmt.astype(np.float64))
    print("   %-32s mean %7.2f  p50 %7.2f  p90 %7.2f  max %7.2f us"
          % ("iteration (same workgroup)", it.mean(), np.median(it),
             np.percentile(it, 90), it.max()))
    polls = s[:, 14]
    print("   look-back polls: mean %.2f  p90 %d  max %d  (>1 poll: %.1f%% of tiles)"
          % (polls.mean(), np.percentile(polls, 90), polls.max(),
             100.0 * (polls > 0).mean()))
    # iteration count per WG
    per_wg = (tiles + grid - 1) // grid
    print("   iterations per WG: %d..%d" % (tiles // grid, per_wg))


def main():
    path = os.environ.get("TRACE_FILE")
    if not path or not os.path.exists(path):
        path = path or os.path.join(tempfile.mkdtemp(), "qhuff.trace")
        os.environ["QHUFF_TRACE"] = path
        import torch
        import qhuff
        n = int(os.environ.get("N", 1 << 20))
        data, off = qhuff.synth_batch(n, max_len=int(os.environ.get("MAXLEN", 64)))
        dev = torch.device("cuda", 0)
        d = torch.from_numpy(data).to(dev)
        o = torch.from_numpy(off.view(np.int32)).to(dev)
        c = qhuff.Codec(0)
        for _ in range(3):
            h, ho = c.encode(d, o, 0)
            r, ro, st = c.decode(h, ho)
        torch.cuda.synchronize()
        assert c.device_error() == 0
        c.close()
    recs = read(path)
    last = {}
    for r in recs:
        last[r[0]] = r
    for k in sorted(last):
        report(*last[k])


if __name__ == "__main__":
    main()
