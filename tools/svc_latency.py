"""Per-call latency of small batches -- the reference's call pattern (a
header block of a few dozen literals) -- through each path:

  svc      qhuff_svc_encode / _decode (resident kernel, pinned request slots)
  host     qhuff_*_batch_host on a context without a service (launch +
           copies + synchronisation per call)
  device   qhuff_*_batch on device buffers + stream synchronise (launch +
           synchronisation per call)
  cpu      the oracle restatement of the reference's loops, one thread

and the service's throughput with T calling threads.  Prints one JSON object.
usage: python tools/svc_latency.py [calls_per_case]"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
    import numpy as np
    import torch
    import qhuff
    import oracle_lib as O

    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    res = {"calls": calls, "cases": {}}
    shapes = [("1 string", 1), ("header block, 20 strings", 20),
              ("64 strings", 64), ("1024 strings", 1024)]
    plain = qhuff.Codec(0)               # no service: host / device paths
    sc = qhuff.Codec(0)
    svc = sc.service()
    dev = torch.device("cuda", 0)
    for name, n in shapes:
        data, off = qhuff.synth_batch(n, seed=17 + n)
        huff, hoff = O.encode_batch(data, off, 0)
        case = {"n": n, "raw_bytes": int(off[-1]), "huff_bytes": int(hoff[-1])}
        k = calls if n <= 64 else max(200, calls // 5)
        eo = np.zeros(qhuff.encode_bound(int(off[-1]), n, 0), np.uint8)
        eoo = np.zeros(n + 1, np.uint32)
        do = np.zeros(qhuff.decode_bound(int(hoff[-1]), n), np.uint8)
        doo = np.zeros(n + 1, np.uint32)
        dst = np.zeros(n, np.uint8)
        d_in = torch.from_numpy(data).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_h = torch.from_numpy(huff).to(dev)
        d_hoff = torch.from_numpy(hoff.view(np.int32)).to(dev)
        d_eo = torch.empty(len(eo), dtype=torch.uint8, device=dev)
        d_eoo = torch.empty(n + 1, dtype=torch.int32, device=dev)
        d_do = torch.empty(len(do), dtype=torch.uint8, device=dev)
        d_doo = torch.empty(n + 1, dtype=torch.int32, device=dev)
        d_st = torch.empty(n, dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream()

        paths = {
            "svc": (lambda: svc.encode(data, off, 0, eo, eoo),
                    lambda: svc.decode(huff, hoff, do, doo, dst)),
            "host": (lambda: plain.encode_host(data, off, 0, eo, eoo),
                     lambda: plain.decode_host(huff, hoff, do, doo, dst)),
            "device": (lambda: (plain.encode_into(d_in, d_off, n, 0, d_eo,
                                                  d_eoo, stream),
                                stream.synchronize()),
                       lambda: (plain.decode_into(d_h, d_hoff, n, d_do, d_doo,
                                                  d_st, stream),
                                stream.synchronize())),
            "cpu": (lambda: O.encode_batch(data, off, 0),
                    lambda: O.decode_batch(huff, hoff)),
        }
        for pname, (fe, fd) in paths.items():
            for op, f in (("encode", fe), ("decode", fd)):
                for _ in range(20):
                    f()
                t = []
                for _ in range(k):
                    a = time.perf_counter()
                    f()
                    t.append((time.perf_counter() - a) * 1e6)
                case["%s_%s_us" % (pname, op)] = {
                    "p50": round(pct(t, 0.5), 2), "p90": round(pct(t, 0.9), 2),
                    "p99": round(pct(t, 0.99), 2)}
        # parity of the service's last outputs
        o_out, o_off = O.encode_batch(data, off, 0)
        e_out, e_off = svc.encode(data, off, 0)
        d_out, d_off2, st = svc.decode(huff, hoff)
        case["svc_bit_exact"] = bool(np.array_equal(e_out, o_out)
                                     and np.array_equal(e_off, o_off)
                                     and bytes(d_out) == bytes(data)
                                     and not st.any())
        res["cases"][name] = case
        print(json.dumps({name: case}), file=sys.stderr, flush=True)

    # throughput: T threads, each calling the service with header blocks
    data, off = qhuff.synth_batch(20, seed=5)
    tp = {}
    for T in (1, 2, 4, 8, 12):
        per = 3000 // T
        done = []

        def worker():
            eo = np.zeros(qhuff.encode_bound(int(off[-1]), 20, 0), np.uint8)
            eoo = np.zeros(21, np.uint32)
            for _ in range(per):
                svc.encode(data, off, 0, eo, eoo)
            done.append(per)

        th = [threading.Thread(target=worker) for _ in range(T)]
        a = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - a
        tp[str(T)] = {"calls_per_s": round(sum(done) / dt),
                      "blocks_per_s": round(sum(done) / dt),
                      "strings_per_s": round(20 * sum(done) / dt)}
    res["svc_threads_header_block_encode"] = tp
    res["svc_stats"] = dict(zip(("served", "launches", "fallbacks"),
                                svc.stats()))
    svc.close()
    sc.close()
    plain.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
