"""Probe of the PCIe-inclusive host path: qhuff_*_batch_host at several
copy-worker counts, next to raw pinned H2D / D2H rates and a plain host
memcpy rate on the same box (one JSON line per measurement)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(threads, shift=21):
    os.environ["QHUFF_HOST_THREADS"] = str(threads)
    os.environ["QHUFF_HOST_CHUNK_SHIFT"] = str(shift)
    sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
    import numpy as np
    import qhuff
    c = qhuff.Codec(0)
    data, off = qhuff.synth_batch(1 << 20)
    raw = int(off[-1])
    h, ho = c.encode_host(data, off, 0)
    h = h.copy()
    # reused, faulted-in result buffers (a fresh np.zeros of the bound
    # costs page faults on first touch -- not the library's time)
    eo = np.ones(qhuff.encode_bound(raw, len(off) - 1, 0), dtype=np.uint8)
    eoo = np.ones(len(off), dtype=np.uint32)
    do = np.ones(qhuff.decode_bound(len(h), len(off) - 1), dtype=np.uint8)
    doo = np.ones(len(off), dtype=np.uint32)
    dst = np.ones(len(off), dtype=np.uint8)
    c.decode_host(h, ho, do, doo, dst)
    te = td = 1e9
    for _ in range(5):
        t = time.perf_counter(); c.encode_host(data, off, 0, eo, eoo)
        te = min(te, time.perf_counter() - t)
        t = time.perf_counter(); c.decode_host(h, ho, do, doo, dst)
        td = min(td, time.perf_counter() - t)
    print(json.dumps({"threads": threads, "chunk_shift": shift, "enc_ms": round(te * 1e3, 3),
                      "dec_ms": round(td * 1e3, 3),
                      "enc_gbps": round(raw / te / 1e9, 2),
                      "dec_gbps": round(raw / td / 1e9, 2)}), flush=True)
    c.close()


def raw_rates():
    import numpy as np
    import torch
    n = 64 << 20
    a = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    b = np.ones(n, dtype=np.uint8)
    an = a.numpy()
    for _ in range(2):
        d.copy_(a, non_blocking=True); a.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("h2d", lambda: d.copy_(a, non_blocking=True)),
                     ("d2h", lambda: a.copy_(d, non_blocking=True))):
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        res[name + "_gbps"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
    t = time.perf_counter()
    for _ in range(5):
        np.copyto(an, b)
    res["memcpy_1thread_gbps"] = round(5 * n / (time.perf_counter() - t) / 1e9, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(int(sys.argv[1]), int(sys.argv[2]))
    else:
        raw_rates()
        for t, sh in ((1, 21), (8, 21), (8, 22), (2, 23), (4, 23), (8, 23),
                      (4, 24), (8, 24), (4, 25)):
            subprocess.check_call([sys.executable, __file__, str(t), str(sh)])
