#!/usr/bin/env python3
"""Small-batch crossover: at what batch size does a GPU
launch beat the CPU per-string path?

For batch sizes 64 .. 1M strings (the bench's synthetic header strings,
U[8,64] B), one synchronous call each way:
  device  encode_into / decode_into on device-resident buffers + stream sync
          (launch + kernel + completion latency; what a caller with data
          already in HBM waits)
  host    encode_host / decode_host: host buffers in and out (PCIe copies
          included; what a patched lsqpack.c batch call waits)
  cpu     the oracle restatement of lsqpack_enc_enc_str(7, ..) /
          lsqpack_huff_decode per string, 1 thread (the reference codes one
          string per call on the connection's thread)
Median of --reps calls after warm-up.  Writes JSON (--out) and prints a
table.  Run on the GPU box:  python tools/crossover.py --out gpurun_out/x.json
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def med(f, reps):
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--max-log2", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import qhuff
    import oracle_lib as O

    codec = qhuff.Codec(0)
    st = torch.cuda.current_stream()
    rows = []
    sizes = [1 << k for k in range(6, a.max_log2 + 1, 2)]
    for n in sizes:
        data, off = qhuff.synth_batch(n, seed=n)
        raw = int(off[-1])
        d = torch.from_numpy(data).cuda()
        o = torch.from_numpy(off.view(np.int32)).cuda()
        eo = torch.empty(qhuff.encode_bound(raw, n, 0), dtype=torch.uint8,
                         device="cuda")
        eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
        codec.encode_into(d, o, n, 0, eo, eoo, st)
        torch.cuda.synchronize()
        hb = int(eoo[-1].item())
        h = eo[:hb].clone()
        ho = eoo.clone()
        h_np = h.cpu().numpy()
        ho_np = ho.cpu().numpy().view(np.uint32)
        do = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8,
                         device="cuda")
        doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
        dst = torch.empty(n, dtype=torch.uint8, device="cuda")
        reps = a.reps if n < (1 << 18) else max(5, a.reps // 4)

        def dev_enc():
            codec.encode_into(d, o, n, 0, eo, eoo, st)
            st.synchronize()

        def dev_dec():
            codec.decode_into(h, ho, n, do, doo, dst, st)
            st.synchronize()

        he = np.ones(qhuff.encode_bound(raw, n, 0), dtype=np.uint8)
        heo = np.ones(n + 1, dtype=np.uint32)
        hd = np.ones(qhuff.decode_bound(hb, n), dtype=np.uint8)
        hdo = np.ones(n + 1, dtype=np.uint32)
        hds = np.ones(n, dtype=np.uint8)

        def host_enc():
            codec.encode_host(data, off, 0, he, heo)

        def host_dec():
            codec.decode_host(h_np, ho_np, hd, hdo, hds)

        for f in (dev_enc, dev_dec, host_enc, host_dec):
            f()
            f()
        r = {"strings": n, "raw_bytes": raw, "huff_bytes": hb,
             "dev_enc_us": med(dev_enc, reps) * 1e6,
             "dev_dec_us": med(dev_dec, reps) * 1e6,
             "host_enc_us": med(host_enc, reps) * 1e6,
             "host_dec_us": med(host_dec, reps) * 1e6,
             "cpu_enc_us": min(O.bench_pass(data, off, 0, 1)
                               for _ in range(3)) * 1e6,
             "cpu_dec_us": min(O.bench_pass(h_np, ho_np, 1, 1)
                               for _ in range(3)) * 1e6}
        ok = (np.array_equal(hdo, off) and not hds.any()
              and np.array_equal(hd[:raw], data))
        r["host_roundtrip_ok"] = bool(ok)
        rows.append(r)
        print("%8d  dev %8.1f %8.1f  host %9.1f %9.1f  cpu1 %10.1f %10.1f us"
              % (n, r["dev_enc_us"], r["dev_dec_us"], r["host_enc_us"],
                 r["host_dec_us"], r["cpu_enc_us"], r["cpu_dec_us"]),
              flush=True)

    def cross(path, op):
        for r in rows:
            if r["%s_%s_us" % (path, op)] < r["cpu_%s_us" % op]:
                return r["strings"]
        return None

    res = {"rows": rows, "device": torch.cuda.get_device_name(0),
           "crossover_strings": {"%s_%s" % (p, op): cross(p, op)
                                 for p in ("dev", "host")
                                 for op in ("enc", "dec")},
           "note": "median synchronous call latency; cpu = oracle per-string "
                   "loop on 1 thread"}
    print(json.dumps(res["crossover_strings"]))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    codec.close()


if __name__ == "__main__":
    main()
