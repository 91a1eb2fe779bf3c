#!/usr/bin/env python3
"""Diagnostic: decode a random batch on the GPU and print the first strings
whose status / bytes differ from the oracle."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import numpy as np
import torch
import oracle_lib as O
import qhuff


def main():
    alpha = {"all": bytes(range(256)), "token": qhuff.TOKEN_ALPHABET,
             "high": bytes(range(128, 256))}[sys.argv[1] if len(sys.argv) > 1 else "all"]
    rng = random.Random(len(alpha))
    strs = [bytes(rng.choice(alpha) for _ in range(rng.randint(0, 80)))
            for _ in range(3000)]
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strs], out=off[1:])
    data = np.frombuffer(b"".join(strs), dtype=np.uint8).copy()
    h, ho = O.encode_batch(data, off, 0)
    c = qhuff.Codec(0)
    dev = torch.device("cuda", 0)
    out, oo, st = c.decode(torch.from_numpy(h).to(dev),
                           torch.from_numpy(ho.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    oo = oo.cpu().numpy().view(np.uint32)
    out = out.cpu().numpy()
    st = st.cpu().numpy()
    print("device_error", c.device_error(), "total", oo[-1], "expect", off[-1])
    bad = 0
    for i, s in enumerate(strs):
        g = bytes(out[oo[i]:oo[i + 1]])
        if st[i] != 0 or g != s:
            bad += 1
            if bad <= 8:
                hs = bytes(h[ho[i]:ho[i + 1]])
                print(i, "tile", i // 256, "len", len(s), "st", st[i],
                      "\n  want", s.hex(), "\n  got ", g.hex(), "\n  huff", hs.hex())
    print("mismatches", bad, "of", len(strs))


if __name__ == "__main__":
    main()
