"""Wall time per bench step (encode + decode of the 1M-string batch) with
the per-launch dispatch-stamped timing on and off, alternating blocks of
steps in one process: what the bench's kernel timing costs the step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np
import torch
import qhuff


def main():
    n = 1 << 20
    dev = torch.device("cuda", 0)
    data, off = qhuff.synth_batch(n, seed=0x9E3779B97F4A7C15)
    codec = qhuff.Codec(0)
    st = torch.cuda.current_stream()
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int32)).to(dev)
    eo = torch.empty(qhuff.encode_bound(len(data), n), dtype=torch.uint8, device=dev)
    eoo = torch.empty(n + 1, dtype=torch.int32, device=dev)
    codec.encode_into(d, o, n, 0, eo, eoo, st)
    torch.cuda.synchronize()
    hb = int(eoo[-1].item())
    h = eo[:hb].clone()
    ho = eoo.clone()
    do = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8, device=dev)
    doo = torch.empty(n + 1, dtype=torch.int32, device=dev)
    ds = torch.empty(n, dtype=torch.uint8, device=dev)

    def block(timed, k=50):
        codec.timing(timed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            codec.encode_into(d, o, n, 0, eo, eoo, st)
            codec.decode_into(h, ho, n, do, doo, ds, st)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / k * 1e6
        if timed:
            codec.timing_read()
        codec.timing(False)
        return t
    for _ in range(3):
        block(False, 10)
    on, off_ = [], []
    for r in range(8):
        if r % 2:
            on.append(block(True)); off_.append(block(False))
        else:
            off_.append(block(False)); on.append(block(True))
    print("us/step timing on  median %.1f  %s" % (np.median(on), [round(x, 1) for x in on]))
    print("us/step timing off median %.1f  %s" % (np.median(off_), [round(x, 1) for x in off_]))
    codec.close()


if __name__ == "__main__":
    main()
