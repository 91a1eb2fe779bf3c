"""qhuff_fastwalk.h (the host replay of huff_decode_fast's stopping point,
lsqpack.c:5243-5466) against the oracle's restatement of the reference
decoder, on the CPU: for every string and every dst_len, the walk's stop
(END_DST at a byte boundary, or the nibble decoder from the byte the walk
names) reproduces oq_huff_decode's (status, n_dst, n_src).  The GPU side of
the shim is tests/test_lsqpack_shim.py."""
import ctypes as C
import json
import os
import random
import subprocess

import pytest

import _paths  # noqa: F401
import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "c", "fastwalk_capi.cpp")
SO = os.path.join(HERE, "c", "_build", "libfastwalk.so")
HDR = os.path.join(os.path.dirname(HERE), "ls-qpack_amd", "csrc",
                   "qhuff_fastwalk.h")

SHORT = b"0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJ-./:=_ %"
MID = b"!\"#$&'()*+,;<>?@[\\]^`{|}~"
LONG = bytes(range(0, 32)) + bytes(range(128, 256))


@pytest.fixture(scope="module")
def walk():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    if (not os.path.exists(SO) or os.path.getmtime(SO)
            < max(os.path.getmtime(SRC), os.path.getmtime(HDR))):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror",
                               "-shared", "-fPIC", "-o", SO, SRC])
    L = C.CDLL(SO)
    L.qh_fast_walk.restype = None
    L.qh_fast_walk.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32,
                               C.c_uint32, C.POINTER(C.c_uint32)]
    lens = [O.code_of(s)[1] for s in range(256)]

    def run(plain, enc, dst_len):
        ln = bytes(lens[b] for b in plain)
        out = (C.c_uint32 * 3)()
        L.qh_fast_walk(ln, len(plain), len(enc), dst_len, out)
        end, n_dst, n_src = out
        if end == 0:
            return O.OK, n_dst, n_src
        if end == 1:
            return O.END_DST, n_dst, n_src
        rest = enc[n_src:]
        s = C.create_string_buffer(rest, len(rest) + 1)
        d = C.create_string_buffer(max(dst_len - n_dst, 1))
        st = O.DecState(0, 0, 0)
        rv = O.lib().oq_huff_decode_full(s, len(rest), d, dst_len - n_dst,
                                         C.byref(st), 1)
        if rv.status in (O.OK, O.END_DST):
            return rv.status, rv.n_dst + n_dst, rv.n_src + n_src
        return rv.status, rv.n_dst, rv.n_src
    return run


def oracle(enc, dst_len):
    s = C.create_string_buffer(enc, len(enc) + 1)
    d = C.create_string_buffer(max(dst_len, 1))
    st = O.DecState(0, 0, 0)
    rv = O.lib().oq_huff_decode(s, len(enc), d, dst_len, C.byref(st), 1)
    return rv.status, rv.n_dst, rv.n_src


def _check(walk, plain):
    enc = O.huffman_enc(plain)
    for dst_len in range(0, len(plain) + 3):
        assert walk(plain, enc, dst_len) == oracle(enc, dst_len), \
            (plain, dst_len)


def test_walk_kats(walk):
    kat = json.load(open(os.path.join(HERE, "golden",
                                      "kat_huff_decode.json")))
    for k in kat["decode_ok"]:
        _check(walk, bytes.fromhex(k["plain"]))


@pytest.mark.parametrize("alpha,lo,hi,n", [
    (SHORT, 0, 60, 150), (SHORT + MID, 1, 60, 150),
    (SHORT + MID + LONG, 1, 40, 150), (LONG, 1, 12, 100),
    (b"e", 1, 40, 40), (bytes(range(256)), 1, 300, 20)])
def test_walk_random(walk, alpha, lo, hi, n):
    rng = random.Random(len(alpha) * 1000 + hi)
    for _ in range(n):
        _check(walk, bytes(rng.choice(alpha)
                           for _ in range(rng.randint(lo, hi))))


def _invalid_inputs(seed):
    """Invalid complete strings of every D3 kind: the EOS code after a
    prefix (short and long codes before it), padding of 8-23 ones, padding
    that is not all ones, random bytes."""
    rng = random.Random(seed)
    eos = "1" * 30
    out = []

    def bits(s):
        return "".join(format(O.code_of(b)[0], "0%db" % O.code_of(b)[1])
                       for b in s)

    def tob(b):
        b += "1" * (-len(b) % 8)
        return int(b, 2).to_bytes(len(b) // 8, "big")
    for _ in range(60):
        s = bytes(rng.choice(SHORT + MID + LONG) for _ in
                  range(rng.randint(0, 30)))
        t = bytes(rng.choice(SHORT) for _ in range(rng.randint(0, 6)))
        out.append(tob(bits(s) + eos + bits(t)))                 # EOS
        out.append(tob(bits(s) + "1" * rng.randint(8, 23)))      # long padding
        pad = "".join(rng.choice("01") for _ in range(rng.randint(1, 7)))
        if "0" in pad:
            b = bits(s) + pad
            if len(b) % 8 == 0:
                out.append(int(b, 2).to_bytes(len(b) // 8, "big"))
            else:
                b += "1" * (-len(b) % 8)
                out.append(int(b, 2).to_bytes(len(b) // 8, "big"))
    for _ in range(300):
        out.append(bytes(rng.randrange(256) for _ in range(rng.randint(1, 14))))
    return [x for x in out if O.huff_decode(x)[0] == O.ERROR]


def test_walk_invalid_every_dst_len(walk_invalid):
    """fast_walk_invalid (the shim's replay for a string the GPU rejected)
    over the symbols decoded before the error reproduces oq_huff_decode's
    (status, n_dst, n_src) at every dst_len: ERROR, or END_DST where dst runs
    out first, or the nibble decoder's result from the byte it names."""
    inputs = _invalid_inputs(21)
    assert len(inputs) > 200
    for enc in inputs:
        for dst_len in range(0, 8 * len(enc) // 5 + 3):
            assert walk_invalid(enc, dst_len) == oracle(enc, dst_len), \
                (enc.hex(), dst_len)


@pytest.fixture(scope="module")
def walk_invalid(walk):
    L = C.CDLL(SO)
    L.qh_fast_walk_invalid.restype = None
    L.qh_fast_walk_invalid.argtypes = [C.c_char_p, C.c_uint32, C.c_char_p,
                                       C.c_uint32, C.c_uint32,
                                       C.POINTER(C.c_uint32)]
    lens = [O.code_of(s)[1] for s in range(256)]

    def run(enc, dst_len):
        prefix, eos = O.decoded_prefix(enc)
        ln = bytes([lens[b] for b in prefix] + ([30] if eos else []))
        out = (C.c_uint32 * 3)()
        L.qh_fast_walk_invalid(ln, len(ln), enc, len(enc), dst_len, out)
        end, n_dst, n_src = out
        if end == 0:
            return O.ERROR, 0, 0
        if end == 1:
            return O.END_DST, n_dst, n_src
        rest = enc[n_src:]
        s = C.create_string_buffer(rest, len(rest) + 1)
        d = C.create_string_buffer(max(dst_len - n_dst, 1))
        st = O.DecState(0, 0, 0)
        rv = O.lib().oq_huff_decode_full(s, len(rest), d, dst_len - n_dst,
                                         C.byref(st), 1)
        if rv.status in (O.OK, O.END_DST):
            return rv.status, rv.n_dst + n_dst, rv.n_src + n_src
        return rv.status, rv.n_dst, rv.n_src
    return run
