"""Header hashing: XXH32 of names and values the way
lsqpack.c:1681-1685 / 3268-3269 / 3308-3309 computes them.

CPU: the oracle restatement (oracle/xxh32_oracle.c) against the golden
vectors produced by the REFERENCE's own deps/xxhash/xxhash.c
(tests/golden/make_xxh32_golden.py), and against that compiled reference
directly when oracle/_ref/libxxh32_ref.so is present.
GPU: qhuff_xxh32_headers / qhuff_xxh32_batch through the C-ABI against the
golden vectors and the oracle; bit-exact."""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_SO = os.path.join(O.ROOT, "oracle", "_ref", "libxxh32_ref.so")

with open(os.path.join(G, "xxh32.json")) as f:
    GOLD = json.load(f)


def pack_headers(pairs):
    parts = []
    for n, v in pairs:
        parts += [n, v]
    off = np.zeros(len(parts) + 1, dtype=np.uint32)
    np.cumsum([len(p) for p in parts], out=off[1:])
    data = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return data, off


def gold_pairs():
    hs = GOLD["headers"]
    pairs = [(bytes.fromhex(h["name"]), bytes.fromhex(h["value"])) for h in hs]
    return (pairs, np.array([h["name_hash"] for h in hs], dtype=np.uint32),
            np.array([h["nameval_hash"] for h in hs], dtype=np.uint32))


# ---- CPU: oracle pinned to the reference ---------------------------------

def test_oracle_matches_reference_strings():
    assert O.xxh32(b"", 0) == 0x02CC5D05          # published XXH32("", 0)
    for v in GOLD["strings"]:
        assert O.xxh32(bytes.fromhex(v["hex"]), v["seed"]) == v["xxh32"]


def test_oracle_matches_reference_headers():
    pairs, h1, h2 = gold_pairs()
    data, off = pack_headers(pairs)
    o1, o2 = O.xxh32_headers(data, off)
    assert np.array_equal(o1, h1) and np.array_equal(o2, h2)


@pytest.mark.skipif(not os.path.exists(REF_SO),
                    reason="oracle/_ref not built (reference not mounted)")
def test_oracle_differential_vs_compiled_reference():
    L = C.CDLL(REF_SO)
    L.XXH32.restype = C.c_uint
    L.XXH32.argtypes = [C.c_char_p, C.c_size_t, C.c_uint]
    rng = random.Random(7)
    for _ in range(3000):
        s = bytes(rng.randrange(256) for _ in range(rng.randrange(200)))
        seed = rng.randrange(1 << 32)
        assert O.xxh32(s, seed) == L.XXH32(s, len(s), seed)


# ---- GPU: the HIP kernel through the C-ABI --------------------------------

def _codec():
    import torch
    import qhuff
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    return qhuff.Codec(0)


@pytest.fixture(scope="module")
def codec():
    c = _codec()
    yield c
    c.close()


def gpu_headers(codec, data, off, seed=O.XXH_SEED, pad_front=0):
    import torch
    d = torch.zeros(len(data) + pad_front + 16, dtype=torch.uint8,
                    device="cuda")
    if len(data):
        d[pad_front:pad_front + len(data)] = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64) + pad_front).to(
        torch.int32).cuda()
    h1, h2 = codec.xxh32_headers(d, o, seed)
    torch.cuda.synchronize()
    return (h1.cpu().numpy().view(np.uint32),
            h2.cpu().numpy().view(np.uint32))


@pytest.mark.gpu
def test_gpu_headers_golden(codec):
    pairs, h1, h2 = gold_pairs()
    data, off = pack_headers(pairs)
    for pad in (0, 3):
        g1, g2 = gpu_headers(codec, data, off, pad_front=pad)
        assert np.array_equal(g1, h1) and np.array_equal(g2, h2)


@pytest.mark.gpu
def test_gpu_strings_golden(codec):
    import torch
    by_seed = {}
    for v in GOLD["strings"]:
        by_seed.setdefault(v["seed"], []).append(v)
    for seed, vs in by_seed.items():
        strs = [bytes.fromhex(v["hex"]) for v in vs]
        off = np.zeros(len(strs) + 1, dtype=np.uint32)
        np.cumsum([len(s) for s in strs], out=off[1:])
        data = np.frombuffer(b"".join(strs) + b"\0" * 16, dtype=np.uint8)
        h = codec.xxh32(torch.from_numpy(data.copy()).cuda(),
                        torch.from_numpy(off.view(np.int32)).cuda(), seed)
        torch.cuda.synchronize()
        want = np.array([v["xxh32"] for v in vs], dtype=np.uint32)
        assert np.array_equal(h.cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["synthetic", "ragged", "long", "empty"])
def test_gpu_headers_random(codec, kind):
    import qhuff
    rng = random.Random(hash(kind) & 0xffff)
    if kind == "synthetic":                     # bench shape: 8..64 B strings
        data, off = qhuff.synth_batch(200001 * 2, seed=99)
    else:
        if kind == "ragged":
            lens = [rng.choice([0, 1, 3, 4, 15, 16, 17, 31, 32, 33, 200])
                    for _ in range(2 * 3001)]
        elif kind == "long":                    # tiles larger than the stage
            lens = [rng.randrange(0, 700) for _ in range(2 * 700)]
        else:
            lens = [0] * (2 * 130)
        blob = bytes(rng.randrange(256) for _ in range(sum(lens)))
        off = np.zeros(len(lens) + 1, dtype=np.uint32)
        np.cumsum(lens, out=off[1:])
        data = np.frombuffer(blob, dtype=np.uint8).copy()
    g1, g2 = gpu_headers(codec, data, off)
    o1, o2 = O.xxh32_headers(data, off)
    assert np.array_equal(g1, o1) and np.array_equal(g2, o2)


@pytest.mark.gpu
def test_gpu_headers_several_rounds(codec):
    """1M headers (16,384 tiles): more tiles than the resident grid has
    waves, so each persistent wave hashes two or three tiles through its
    prefetch loop (the synthetic case above fits one round)"""
    import qhuff
    data, off = qhuff.synth_batch(2 * (1 << 20), seed=123)
    g1, g2 = gpu_headers(codec, data, off)
    o1, o2 = O.xxh32_headers(data, off)
    assert np.array_equal(g1, o1) and np.array_equal(g2, o2)


@pytest.mark.gpu
def test_gpu_zero_headers(codec):
    g1, g2 = gpu_headers(codec, np.zeros(0, dtype=np.uint8),
                         np.zeros(1, dtype=np.uint32))
    assert len(g1) == 0 and len(g2) == 0


@pytest.mark.gpu
def test_gpu_headers_host_path(codec):
    pairs, h1, h2 = gold_pairs()
    data, off = pack_headers(pairs)
    pad = 7                                     # off[0] != 0
    data2 = np.concatenate([np.zeros(pad, np.uint8), data])
    g1, g2 = codec.xxh32_headers_host(data2, off + pad)
    assert np.array_equal(g1, h1) and np.array_equal(g2, h2)
