"""Probe: encode and decode of a bench step on two streams (two contexts, so
two sets of look-back flags) vs one stream.  A kernel's grid is exactly the
co-resident waves, so the two kernels only share the GPU where one's last,
partly busy round frees CUs for the other's first.  Prints step times; the
bench itself stays single-stream.  Usage: python tools/overlap_probe.py"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
import qhuff  # noqa: E402


def main():
    n, copies, steps = 1 << 20, 4, 50
    data, off = qhuff.synth_batch(n)
    raw = int(off[-1])
    ca, cb = qhuff.Codec(0), qhuff.Codec(0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    d_in = [torch.from_numpy(data).cuda() for _ in range(copies)]
    d_off = [torch.from_numpy(off.view(np.int32)).cuda() for _ in range(copies)]
    cap = qhuff.encode_bound(raw, n, 0)
    e_out = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(copies)]
    e_off = [torch.empty(n + 1, dtype=torch.int32, device="cuda") for _ in range(copies)]
    h, ho = ca.encode(d_in[0], d_off[0], 0)
    torch.cuda.synchronize()
    hb = int(ho.cpu().numpy().view(np.uint32)[-1])
    d_h = [h[:hb].clone() for _ in range(copies)]
    d_ho = [ho.clone() for _ in range(copies)]
    dcap = qhuff.decode_bound(hb, n)
    d_out = [torch.empty(dcap, dtype=torch.uint8, device="cuda") for _ in range(copies)]
    d_oo = [torch.empty(n + 1, dtype=torch.int32, device="cuda") for _ in range(copies)]
    d_st = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(copies)]

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
           for _ in range(steps)]

    def run(two, null, ev):
        s0 = torch.cuda.current_stream() if null else sa
        s1 = sb if two else s0
        for i in range(steps):
            k, j = i % copies, (i + copies // 2) % copies
            if ev:
                evs[i][0].record(s0)
            ca.encode_into(d_in[k], d_off[k], n, 0, e_out[k], e_off[k], s0)
            if ev:
                evs[i][1].record(s0)
            cb.decode_into(d_h[j], d_ho[j], n, d_out[j], d_oo[j], d_st[j], s1)
            if ev:
                evs[i][2].record(s1)

    cases = [(False, False, False), (True, False, False),
             (False, True, False), (False, True, True), (False, False, True)]
    for two, null, ev in cases + cases:
        run(two, null, ev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(two, null, ev)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) * 1e6 / steps
        ok = (torch.equal(d_out[0][:raw], d_in[0]) and not d_st[0].any()
              and ca.device_error() == 0 and cb.device_error() == 0)
        kern = ""
        if ev:
            e = sum(x[0].elapsed_time(x[1]) for x in evs) * 1e3 / steps
            d = sum(x[1].elapsed_time(x[2]) for x in evs) * 1e3 / steps
            kern = "  events: enc %.1f dec %.1f us" % (e, d)
        print("%s %s %s  %.1f us/step  %.1f GB/s enc+dec  ok=%s%s"
              % ("two-streams" if two else "one-stream ",
                 "null-stream" if null else "own-stream ",
                 "events   " if ev else "no-events", us,
                 2 * raw / us / 1e3, ok, kern), flush=True)
    ca.close()
    cb.close()


if __name__ == "__main__":
    main()
