#!/usr/bin/env python3
"""Encode and decode of the bench batch (1M strings each) run sequentially on
one stream vs concurrently on two streams (two contexts), per step, with the
library in QHUFF_LIB (e.g. a build with fewer waves per workgroup, so that an
encode and a decode workgroup fit on one CU together).  Prints ms per step and
checks both outputs against a sequential reference pass."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np
import torch
import qhuff


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    steps = 50
    dev = torch.device("cuda", 0)
    data, off = qhuff.synth_batch(n)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int32)).to(dev)
    ce, cd = qhuff.Codec(0), qhuff.Codec(0)
    h, ho = ce.encode(d, o, 0)
    torch.cuda.synchronize()
    hb = int(ho[-1].item())
    h = h[:hb].clone()
    e_out = torch.empty(qhuff.encode_bound(len(data), n), dtype=torch.uint8, device=dev)
    e_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_out = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()

    def seq():
        ce.encode_into(d, o, n, 0, e_out, e_off, s1)
        cd.decode_into(h, ho, n, d_out, d_off, st, s1)

    def conc():
        ev = torch.cuda.Event()
        ev.record(s1)
        s2.wait_event(ev)
        ce.encode_into(d, o, n, 0, e_out, e_off, s1)
        cd.decode_into(h, ho, n, d_out, d_off, st, s2)
        ev2 = torch.cuda.Event()
        ev2.record(s2)
        s1.wait_event(ev2)

    for name, fn in (("sequential", seq), ("concurrent", conc),
                     ("sequential", seq), ("concurrent", conc)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s1)
        for _ in range(steps):
            fn()
        b.record(s1)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / steps
        ok = (bool(torch.equal(e_out[:hb], h)) and bool(torch.equal(e_off, ho))
              and bool(torch.equal(d_out[:len(data)], d)) and not bool(st.any())
              and ce.device_error() == 0 and cd.device_error() == 0)
        gbps = 2 * len(data) / (ms * 1e-3) / 1e9
        print("%-11s %.4f ms/step  %.1f GB/s enc+dec  ok=%s" % (name, ms, gbps, ok),
              flush=True)


if __name__ == "__main__":
    main()
