"""A second, independent pin of the oracle: nghttp2's HPACK Huffman coder.

SURVEY.md 8(c) recovered the RFC 7541 code from libnghttp2 and checked the
reference against nghttp2's inflater.  This CPU test repeats that
differential against the oracle, through the system libnghttp2 (part of the
container image, not of the reference; skipped where it is absent):

* decode: a value literal carrying the oracle's Huffman payload, inside an
  HPACK "literal never indexed, new name" field line, is inflated by
  nghttp2_hd_inflate_hd2 to the original string; random payloads are
  rejected by nghttp2 exactly when the oracle rejects them (D3);
* encode: nghttp2_hd_deflate_hd's value literal (H bit, 7-bit-prefix
  length, Huffman when strictly shorter) equals the oracle's
  lsqpack_enc_enc_str(7, ...) byte for byte.
"""
import ctypes as C
import random

import pytest

import _paths  # noqa: F401
import oracle_lib as O

try:
    NG = C.CDLL("libnghttp2.so.14")
except OSError:
    NG = None

pytestmark = pytest.mark.skipif(NG is None, reason="libnghttp2 not installed")


class NV(C.Structure):
    _fields_ = [("name", C.c_void_p), ("value", C.c_void_p),
                ("namelen", C.c_size_t), ("valuelen", C.c_size_t),
                ("flags", C.c_uint8)]


INFLATE_FINAL, INFLATE_EMIT = 0x01, 0x02
NV_FLAG_NO_INDEX = 0x01


def _setup():
    NG.nghttp2_hd_inflate_new.argtypes = [C.POINTER(C.c_void_p)]
    NG.nghttp2_hd_inflate_hd2.restype = C.c_ssize_t
    NG.nghttp2_hd_inflate_hd2.argtypes = [C.c_void_p, C.POINTER(NV),
                                          C.POINTER(C.c_int), C.c_char_p,
                                          C.c_size_t, C.c_int]
    NG.nghttp2_hd_inflate_end_headers.argtypes = [C.c_void_p]
    NG.nghttp2_hd_inflate_del.argtypes = [C.c_void_p]
    NG.nghttp2_hd_deflate_new.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    NG.nghttp2_hd_deflate_hd.restype = C.c_ssize_t
    NG.nghttp2_hd_deflate_hd.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t,
                                         C.POINTER(NV), C.c_size_t]
    NG.nghttp2_hd_deflate_del.argtypes = [C.c_void_p]


if NG is not None:
    _setup()


def prefixed_int(v, prefix, first):
    """HPACK integer with a `prefix`-bit prefix; `first` holds the bits above."""
    m = (1 << prefix) - 1
    if v < m:
        return bytes([first | v])
    out = [first | m]
    v -= m
    while v >= 128:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def nghttp2_inflate_value(huff_payload):
    """Inflate one 'literal never indexed, new name x' field line whose value
    is the Huffman payload; returns the value bytes, or None on error."""
    block = (b"\x10" + prefixed_int(1, 7, 0) + b"x"
             + prefixed_int(len(huff_payload), 7, 0x80) + huff_payload)
    inf = C.c_void_p()
    assert NG.nghttp2_hd_inflate_new(C.byref(inf)) == 0
    try:
        nv, flags = NV(), C.c_int(0)
        pos, got = 0, None
        while True:
            rv = NG.nghttp2_hd_inflate_hd2(inf, C.byref(nv), C.byref(flags),
                                           block[pos:], len(block) - pos, 1)
            if rv < 0:
                return None
            pos += rv
            if flags.value & INFLATE_EMIT:
                got = C.string_at(nv.value, nv.valuelen)
            if flags.value & INFLATE_FINAL:
                NG.nghttp2_hd_inflate_end_headers(inf)
                return got
            if rv == 0 and not (flags.value & INFLATE_EMIT):
                return None
    finally:
        NG.nghttp2_hd_inflate_del(inf)


def nghttp2_value_literal(value):
    """The value literal nghttp2's deflater writes for header x: value."""
    dfl = C.c_void_p()
    assert NG.nghttp2_hd_deflate_new(C.byref(dfl), 0) == 0
    try:
        nm = C.create_string_buffer(b"x-qhuff-test", 12)
        vl = C.create_string_buffer(value, max(len(value), 1))
        nv = NV(C.cast(nm, C.c_void_p), C.cast(vl, C.c_void_p), 12,
                len(value), NV_FLAG_NO_INDEX)
        buf = C.create_string_buffer(4 * len(value) + 64)
        n = NG.nghttp2_hd_deflate_hd(dfl, buf, len(buf), C.byref(nv), 1)
        assert n > 0
        b = buf.raw[:n]
    finally:
        NG.nghttp2_hd_deflate_del(dfl)

    def literal_end(p):
        v, q = b[p] & 0x7F, p + 1
        if v == 0x7F:
            m, sh = 0, 0
            while True:
                m |= (b[q] & 0x7F) << sh
                sh += 7
                q += 1
                if not b[q - 1] & 0x80:
                    break
            v = 0x7F + m
        return q + v

    p = 0
    while b[p] & 0xE0 == 0x20:           # 001xxxxx table size update(s)
        if b[p] & 0x1F == 0x1F:
            p += 1
            while b[p] & 0x80:
                p += 1
        p += 1
    # 0001xxxx never indexed, name index 0 -> name literal, value literal
    assert b[p] == 0x10
    vstart = literal_end(p + 1)
    assert literal_end(vstart) == len(b)
    return b[vstart:]


ALPHABETS = [bytes(range(32, 127)), b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, ",
             bytes(range(256))]


def _strings(seed, n, lo, hi):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        a = ALPHABETS[i % len(ALPHABETS)]
        out.append(bytes(rng.choice(a) for _ in range(rng.randint(lo, hi))))
    return out


def test_nghttp2_inflates_oracle_payloads():
    for s in _strings(1, 600, 0, 90) + [bytes(300), bytes(range(256)) * 2]:
        h = O.huffman_enc(s)
        assert nghttp2_inflate_value(h) == s, s.hex()


def test_nghttp2_rejects_what_the_oracle_rejects():
    rng = random.Random(2)
    agree = rejected = 0
    for _ in range(3000):
        src = bytes(rng.randrange(256) for _ in range(rng.randint(1, 16)))
        st, out = O.huff_decode(src)
        ng = nghttp2_inflate_value(src)
        assert (ng is None) == (st == O.ERROR), src.hex()
        if ng is not None:
            assert ng == out
        agree += 1
        rejected += st == O.ERROR
    assert agree == 3000 and 0 < rejected < 3000


def test_nghttp2_value_literal_equals_enc_enc_str():
    for s in _strings(3, 600, 0, 140):
        assert nghttp2_value_literal(s) == O.enc_enc_str(7, s), s.hex()
