#!/usr/bin/env python3
"""Kernel time vs batch size (tiles per wave): separates fixed per-launch
cost from per-tile cost.  Prints median encode / decode kernel µs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np
import torch
import qhuff


def time_pair(codec, n, reps=20):
    data, off = qhuff.synth_batch(n)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int32)).to(dev)
    h, ho = codec.encode(d, o, 0)
    torch.cuda.synchronize()
    hb = int(ho[-1].item())
    h = h[:hb].clone()
    e_out = torch.empty(qhuff.encode_bound(len(data), n), dtype=torch.uint8, device=dev)
    e_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_out = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8, device=dev)
    d_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    te, td = [], []
    for it in range(reps + 3):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record(s)
        codec.encode_into(d, o, n, 0, e_out, e_off, s)
        e1.record(s)
        codec.decode_into(h, ho, n, d_out, d_off, st, s)
        e2.record(s)
        torch.cuda.synchronize()
        if it >= 3:
            te.append(e0.elapsed_time(e1) * 1e3)
            td.append(e1.elapsed_time(e2) * 1e3)
    return float(np.median(te)), float(np.median(td))


def main():
    codec = qhuff.Codec(0)
    ns = [int(x) for x in sys.argv[1:]] or [64, 4096, 65536, 196608, 393216,
                                            786432, 1048576, 2097152]
    for n in ns:
        e, dd = time_pair(codec, n)
        print("n=%8d tiles=%6d  enc %8.1f us  dec %8.1f us  err %d"
              % (n, (n + 63) // 64, e, dd, codec.device_error()), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
