#!/usr/bin/env python3
"""Regenerate tests/golden/xxh32.json: XXH32 outputs of the REFERENCE's own
deps/xxhash/xxhash.c (compiled where it lies by `make -C oracle ref` into
oracle/_ref/libxxh32_ref.so; run in the build container, where
/root/reference exists).

Vectors:
  * "strings": every length 0..96 over a fixed pseudo-random byte pattern
    (all stripe / 4-byte / 1-byte tail combinations), at seeds 0,
    LSQPACK_XXH_SEED (lsqpack.c:623) and 0x9E3779B1, plus 64 random strings
    of 0..300 bytes;
  * "headers": every distinct (name, value) of the committed QIF corpora
    (tests/golden/data/*.qif) hashed the way lsqpack.c:1681-1685 does:
    name_hash = XXH32(name, LSQPACK_XXH_SEED),
    nameval_hash = XXH32(value, name_hash).
Usage: python tests/golden/make_xxh32_golden.py
"""
import ctypes as C
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import qpack_frames as Q  # noqa: E402

SEED = 39378473
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libxxh32_ref.so")


def main():
    L = C.CDLL(REF_SO)
    L.XXH32.restype = C.c_uint
    L.XXH32.argtypes = [C.c_char_p, C.c_size_t, C.c_uint]
    rng = random.Random(20261016)
    pat = bytes(rng.randrange(256) for _ in range(96))
    strings = []
    for seed in (0, SEED, 0x9E3779B1):
        for n in range(97):
            s = pat[:n]
            strings.append({"hex": s.hex(), "seed": seed,
                            "xxh32": L.XXH32(s, n, seed)})
    for _ in range(64):
        s = bytes(rng.randrange(256) for _ in range(rng.randrange(301)))
        seed = rng.randrange(1 << 32)
        strings.append({"hex": s.hex(), "seed": seed,
                        "xxh32": L.XXH32(s, len(s), seed)})
    headers, seen = [], set()
    for name in sorted(os.listdir(os.path.join(HERE, "data"))):
        if not name.endswith(".qif"):
            continue
        with open(os.path.join(HERE, "data", name), "rb") as f:
            for hl in Q.qif_header_lists(f.read()):
                for n, v in hl:
                    if (n, v) in seen:
                        continue
                    seen.add((n, v))
                    nh = L.XXH32(n, len(n), SEED)
                    headers.append({"name": n.hex(), "value": v.hex(),
                                    "name_hash": nh,
                                    "nameval_hash": L.XXH32(v, len(v), nh)})
    out = {"source": "deps/xxhash/xxhash.c (reference, compiled by "
                     "oracle/Makefile ref) via tests/golden/"
                     "make_xxh32_golden.py",
           "seed": SEED, "strings": strings, "headers": headers}
    with open(os.path.join(HERE, "xxh32.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    import hashlib
    man = os.path.join(HERE, "MANIFEST.sha256")
    with open(os.path.join(HERE, "xxh32.json"), "rb") as f:
        line = "%s  xxh32.json\n" % hashlib.sha256(f.read()).hexdigest()
    with open(man) as f:
        lines = [x for x in f if not x.rstrip().endswith("  xxh32.json")]
    with open(man, "w") as f:
        f.writelines(sorted(lines + [line], key=lambda x: x.split()[1]))
    print("%d strings, %d headers" % (len(strings), len(headers)))


if __name__ == "__main__":
    main()
