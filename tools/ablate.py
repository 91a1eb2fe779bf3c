#!/usr/bin/env python3
"""Kernel-time ablations (QHUFF_DEBUG switches, timing only; outputs are
wrong under any switch).  Prints median kernel µs per variant."""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np
import torch
import qhuff


def main():
    n = int(os.environ.get("N", 1 << 20))
    variants = [int(v, 0) for v in (sys.argv[1:] or ["0", "1", "2", "3", "4",
                                                      "7", "8", "15"])]
    data, off = qhuff.synth_batch(n)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int32)).to(dev)
    base = qhuff.Codec(0)
    h, ho = base.encode(d, o, 0)
    torch.cuda.synchronize()
    hb = int(ho[-1].item())
    h = h[:hb].clone()
    base.close()
    big = 4096 * 65536 + (1 << 24)
    e_out = torch.empty(max(big, qhuff.encode_bound(len(data), n)), dtype=torch.uint8, device=dev)
    e_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_out = torch.empty(max(big, qhuff.decode_bound(hb, n)), dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    res = {}
    for v in variants:
        os.environ["QHUFF_DEBUG"] = str(v)
        c = qhuff.Codec(0)
        s = torch.cuda.current_stream()
        te, td = [], []
        for it in range(25):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(s)
            c.encode_into(d, o, n, 0, e_out, e_off, s)
            e1.record(s)
            c.decode_into(h, ho, n, d_out, d_off, st, s)
            e2.record(s)
            torch.cuda.synchronize()
            if it >= 5:
                te.append(e0.elapsed_time(e1) * 1e3)
                td.append(e1.elapsed_time(e2) * 1e3)
        err = c.device_error()
        if v & 0x40:
            c.debug_clock()
            names = ["claim", "load", "codec", "scan+start", "compact/pack",
                     "lookback", "copyout", "-"]
            tiles = (n + 63) // 64
            for which in ("enc", "dec"):
                for it in range(10):
                    if which == "enc":
                        c.encode_into(d, o, n, 0, e_out, e_off, s)
                    else:
                        c.decode_into(h, ho, n, d_out, d_off, st, s)
                torch.cuda.synchronize()
                cl = c.debug_clock()
                tot = sum(cl)
                print("  %s cycles/tile by phase (wave-cycles): " % which
                      + "  ".join("%s %.0f" % (nm, x / tiles / 10)
                                  for nm, x in zip(names, cl) if x)
                      + "   total %.0f" % (tot / tiles / 10), flush=True)
        c.close()
        res[v] = (float(np.median(te)), float(np.median(td)))
        print("dbg=%#5x  enc %8.1f us   dec %8.1f us  device_error %d"
              % (v, *res[v], err), flush=True)
    os.environ.pop("QHUFF_DEBUG", None)
    print(json.dumps({str(k): v for k, v in res.items()}))


if __name__ == "__main__":
    main()
