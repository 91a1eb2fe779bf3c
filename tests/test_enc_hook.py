"""Encoder-side hook: lsqpack_enc_enc_str
(lsqpack.c:839-876) rebuilt from a precomputed Huffman payload by
qhuff_frame_literal, so a patched lsqpack.c can batch-encode every name and
value of a header list on the GPU first and frame each literal on demand.

CPU: framing (host code) against the reference's test_enc_str.c KATs and the
oracle's lsqpack_enc_enc_str over the QIF corpora and length-prefix
boundaries, incl. dst[0] high bits and short dst_len (-1).
GPU: payloads from one QHUFF_ENC_PAYLOAD batch, framed, equal (a) the oracle
and (b) the literal bytes the reference itself wrote into the interop
streams."""
import json
import os
import random

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O
import qpack_frames as Q
import qhuff

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STREAMS = ["netbsd", "fb-req", "fb-resp"]


def data_file(name):
    with open(os.path.join(G, "data", name), "rb") as f:
        return f.read()


def corpus_strings():
    s = set()
    for name in STREAMS + ["long-codes"]:
        s |= Q.qif_strings(data_file(name + ".qif"))
    return sorted(s)


def test_frame_reference_kats():
    kats = json.load(open(os.path.join(G, "kat_enc_str.json")))["enc_str"]
    for k in kats:
        s = bytes.fromhex(k["str"])
        r = qhuff.frame_literal(k["prefix_bits"], s, O.huffman_enc(s))
        assert r == bytes.fromhex(k["out"]), k["source"]
        assert len(r) == k["retval"]


def test_frame_matches_oracle_enc_enc_str():
    rng = random.Random(3)
    strs = corpus_strings()
    # lengths around every prefix boundary: 2^p - 1, + 127, + 16383
    for n in (6, 7, 8, 30, 31, 32, 126, 127, 128, 129, 134, 135, 158, 159,
              160, 16381, 16382, 16383, 16384, 16390, 16413, 16414):
        strs.append(bytes(rng.choice(b"abcxyz019-_") for _ in range(n)))
        strs.append(bytes(rng.randrange(256) for _ in range(n)))
    for s in strs:
        h = O.huffman_enc(s)
        for p in (3, 5, 7):
            fb = rng.randrange(256)
            want = O.enc_enc_str(p, s, fb)
            assert qhuff.frame_literal(p, s, h, fb) == want
            need = len(want)
            assert qhuff.frame_literal(p, s, h, fb, dst_len=need - 1) == \
                O.enc_enc_str(p, s, fb, dst_len=need - 1) == -1
    assert qhuff.frame_literal(4, b"a", b"\x1f") == -1       # bad prefix


# ---- GPU ---------------------------------------------------------------------

@pytest.fixture(scope="module")
def codec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    c = qhuff.Codec(0)
    yield c
    c.close()


def gpu_payloads(codec, strs):
    import torch
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strs], out=off[1:])
    data = np.frombuffer(b"".join(strs) + b"\0" * 16, dtype=np.uint8).copy()
    out, oo = codec.encode(torch.from_numpy(data).cuda(),
                           torch.from_numpy(off.view(np.int32)).cuda(),
                           qhuff.ENC_PAYLOAD)
    torch.cuda.synchronize()
    oo = oo.cpu().numpy().view(np.uint32)
    ob = out[:int(oo[-1])].cpu().numpy().tobytes()
    return [ob[oo[i]:oo[i + 1]] for i in range(len(strs))]


@pytest.mark.gpu
def test_gpu_payloads_framed_equal_oracle(codec):
    strs = corpus_strings()
    pays = gpu_payloads(codec, strs)
    rng = random.Random(9)
    for s, h in zip(strs, pays):
        for p in (3, 5, 7):
            fb = rng.randrange(256)
            assert qhuff.frame_literal(p, s, h, fb) == O.enc_enc_str(p, s, fb)


@pytest.mark.gpu
def test_gpu_payloads_framed_equal_reference_wire(codec):
    """Every literal of the reference-encoded streams is re-created byte for
    byte from its decoded string and a GPU payload."""
    lits = []
    for name in STREAMS:
        for d in Q.stream_literals(data_file(name + ".out.256.100.1")):
            s = d["payload"]
            if d["huffman"]:
                st, s = O.huff_decode(s)
                assert st == O.OK
            lits.append((d, s))
    pays = gpu_payloads(codec, [s for _, s in lits])
    assert len(lits) > 100
    for (d, s), h in zip(lits, pays):
        got = qhuff.frame_literal(d["prefix_bits"], s, h, d["first_byte"])
        assert got == d["wire"]
