"""In-process A/B of two libqhuff.so builds: one process, one set of device
buffers, the two libraries' kernels timed alternately (blocks of launches,
each launch timed by its own dispatch timestamps (qhuff_timing_*, ABI 4;
HIP events per launch for older libraries), so box-to-box and
process-to-process variance cancel.  Prints per-library median and mean
kernel times for encode and decode of the bench workload (1,048,576 token
strings, 8-64 B), or with WORKLOAD=corpus / alphabet_c of bench.py's
real-workload legs (qhuff/workload.py).

usage: [WORKLOAD=...] python tools/ab_inproc.py LIB_A LIB_B [rounds] [per_block]
(LIB[@VAR=VALUE,...]: knobs set while that context is opened)"""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))


def load(spec):
    # LIB[@VAR=VALUE[,VAR=VALUE...]]: the variables are set while the
    # context is opened (qhuff_open reads its knobs then), so one library
    # can be A/B-ed against itself with other launch knobs
    path, _, envs = spec.partition("@")
    L = C.CDLL(os.path.abspath(path))
    vp = C.c_void_p
    L.qhuff_open.restype = C.c_int
    L.qhuff_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.qhuff_encode_batch.restype = C.c_int
    L.qhuff_encode_batch.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint, vp,
                                     vp, vp]
    L.qhuff_decode_batch.restype = C.c_int
    L.qhuff_decode_batch.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, vp, vp]
    ctx = C.c_void_p()
    saved = {}
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    assert L.qhuff_open(0, C.byref(ctx)) == 0
    for k, v in saved.items():
        if v is None:
            del os.environ[k]
        else:
            os.environ[k] = v
    try:
        L.qhuff_timing_enable.argtypes = [vp, C.c_int]
        L.qhuff_timing_read.argtypes = [vp, vp, vp, C.c_uint32]
        L.timed = True
    except AttributeError:
        L.timed = False
    return L, ctx


def main():
    import numpy as np
    import torch
    import qhuff
    libs = sys.argv[1:3]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    per = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    n = 1 << 20
    dev = torch.device("cuda", 0)
    wl = os.environ.get("WORKLOAD", "synthetic")
    if wl == "corpus":
        from qhuff import workload
        data, off = workload.corpus_batch(
            n, os.path.join(ROOT, "tests", "golden", "data"))
    elif wl == "alphabet_c":
        from qhuff import workload
        data, off = workload.alphabet_c(n)
    else:
        data, off = qhuff.synth_batch(n, seed=0x9E3779B97F4A7C15)
    raw = int(off[-1])
    d_in = torch.from_numpy(data).to(dev)
    d_off = torch.from_numpy(off.view(np.int32)).to(dev)
    codec = qhuff.Codec(0)
    h_out, h_off = codec.encode(d_in, d_off, 0)
    torch.cuda.synchronize()
    hb = int(h_off[-1].item())
    e_out = torch.empty(qhuff.encode_bound(raw, n, 0), dtype=torch.uint8,
                        device=dev)
    e_off = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_out = torch.empty(qhuff.decode_bound(hb, n), dtype=torch.uint8,
                        device=dev)
    d_ooff = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    L = [load(p) for p in libs]

    def enc(k):
        lb, ctx = L[k]
        assert lb.qhuff_encode_batch(ctx, d_in.data_ptr(), d_off.data_ptr(), n,
                                     0, e_out.data_ptr(), e_off.data_ptr(),
                                     sp) == 0

    def dec(k):
        lb, ctx = L[k]
        assert lb.qhuff_decode_batch(ctx, h_out.data_ptr(), h_off.data_ptr(),
                                     n, d_out.data_ptr(), d_ooff.data_ptr(),
                                     d_st.data_ptr(), sp) == 0

    times = {(k, op): [] for k in range(2) for op in ("enc", "dec")}
    for k in range(2):                      # warm both
        for _ in range(5):
            enc(k)
            dec(k)
    torch.cuda.synchronize()
    for r in range(rounds):
        for k in ((0, 1) if r % 2 == 0 else (1, 0)):
            for op, fn in (("enc", enc), ("dec", dec)):
                lb, ctx = L[k]
                if lb.timed:
                    lb.qhuff_timing_enable(ctx, 1)
                    for i in range(per):
                        fn(k)
                    kinds = (C.c_uint32 * per)()
                    us = (C.c_double * per)()
                    m = lb.qhuff_timing_read(ctx, kinds, us, per)
                    lb.qhuff_timing_enable(ctx, 0)
                    times[(k, op)] += [us[i] for i in range(m)]
                    continue
                ev = [torch.cuda.Event(enable_timing=True)
                      for _ in range(per + 1)]
                ev[0].record(stream)
                for i in range(per):
                    fn(k)
                    ev[i + 1].record(stream)
                torch.cuda.synchronize()
                times[(k, op)] += [ev[i].elapsed_time(ev[i + 1]) * 1e3
                                   for i in range(per)]
    ok = (torch.equal(d_out[:raw], d_in) and bool((d_st == 0).all()))
    res = {"ok": ok, "workload": wl, "rounds": rounds, "per_block": per}
    for k, name in enumerate("ab"):
        for op in ("enc", "dec"):
            t = times[(k, op)]
            res["%s_%s_med" % (name, op)] = round(statistics.median(t), 2)
            res["%s_%s_mean" % (name, op)] = round(statistics.mean(t), 2)
    for op in ("enc", "dec"):
        res["%s_b_over_a" % op] = round(res["b_%s_med" % op]
                                        / res["a_%s_med" % op], 4)
    res["libs"] = libs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
