"""Diagnostic for the cooperative long-string decode: decode batches with a
QH_COOP_DEBUG build (QHUFF_LIB) -- a string the wave could not decode comes
back with status 7 and, as its output, the record of its first failing
segment (reason bits: 1 output too big, 2 count mismatch, 4 error in the
write walk, 8 exits do not chain) -- and dump those strings with their
tile's cooperative set.

usage: QHUFF_LIB=.../libqhuff_coopdbg.so python tools/coop_debug.py OUT.json"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import qhuff
    from qhuff import workload as W
    import qpack_frames as Q
    codec = qhuff.Codec(0)
    G = os.path.join(ROOT, "tests", "golden", "data")
    batches = {}
    raw = open(os.path.join(G, "fb-resp.out.256.100.1"), "rb").read()
    lits = [l["payload"] for l in Q.stream_literals(raw) if l["huffman"]]
    off = np.zeros(len(lits) + 1, np.uint32)
    np.cumsum([len(x) for x in lits], out=off[1:])
    batches["fb-resp"] = (np.frombuffer(b"".join(lits), np.uint8).copy(), off)
    d, o = W.corpus_batch(1 << 16, G)
    dd = torch.from_numpy(d).cuda()
    oo = torch.from_numpy(o.view(np.int32)).cuda()
    h, ho = codec.encode(dd, oo, 0)
    torch.cuda.synchronize()
    hoff = ho.cpu().numpy().view(np.uint32).copy()
    batches["corpus64k"] = (h[:int(hoff[-1])].cpu().numpy(), hoff)
    res = {}
    for name, (data, off) in batches.items():
        dt = torch.from_numpy(data).cuda()
        ot = torch.from_numpy(off.view(np.int32)).cuda()
        out, out_off, st = codec.decode(dt, ot)
        torch.cuda.synchronize()
        st = st.cpu().numpy()
        oo = out_off.cpu().numpy().view(np.uint32)
        ob = out.cpu().numpy()
        bad = np.nonzero(st == 7)[0]
        hl = np.diff(off.astype(np.int64))
        ent = {"strings": int(len(off) - 1), "status7": int(len(bad)),
               "other_nonzero": int(((st != 0) & (st != 7)).sum()),
               "cases": []}
        for i in bad[:12]:
            t0 = (i // 64) * 64
            tile_hl = hl[t0:t0 + 64].tolist()
            rec = np.frombuffer(ob[oo[i]:oo[i] + 32].tobytes(),
                                np.uint32).tolist()
            ent["cases"].append({
                "index": int(i), "tile_first": int(t0),
                "record[why,q,m,T,exit,next,S,nseg]": rec,
                "huff_hex": bytes(data[off[i]:off[i + 1]]).hex(),
                "tile_huff_lens": tile_hl})
        res[name] = ent
        print(name, ent["strings"], "status7", ent["status7"],
              "other", ent["other_nonzero"], flush=True)
    json.dump(res, open(sys.argv[1], "w"))


if __name__ == "__main__":
    main()
