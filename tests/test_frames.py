"""Literal-span pre-parse of QPACK wire data + batched literal decode
(include/qhuff.h qhuff_scan_* /
qhuff_decode_literals_host).

CPU: the C scanner in libqhuff.so (host code, no device) finds exactly the
literals the test-side wire reader (tests/qpack_frames.py) finds in the
reference-encoded interop streams and the reference's header-block /
encoder-stream KATs, resumes encoder streams at any split, and rejects what
lsqpack_dec_int / _int24 reject (lsqpack.c:2372-2460).
GPU: every literal of those streams decoded in one batch equals the oracle's
decode and is a name or value of the QIF the reference encoded it from."""
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


def expect(lits_py):
    return [(d["end"] - len(d["payload"]), len(d["payload"]), d["huffman"],
             d["prefix_bits"], d["end"] - len(d["payload"]) - d["start"])
            for d in lits_py]


def got(lits):
    return [(l.pos, l.len, l.huffman, l.prefix_bits, l.hdr_len) for l in lits]


def frames(name):
    return list(Q.read_interop(data_file(name + ".out.256.100.1")))


# ---- CPU: host scanner ------------------------------------------------------

@pytest.mark.parametrize("name", STREAMS)
def test_scan_matches_wire_reader(name):
    n_enc = n_sec = 0
    for sid, payload in frames(name):
        if sid == 0:
            rc, lits, used = qhuff.scan_encoder_stream(payload)
            assert rc == qhuff.OK
            py = []
            for kind, info in Q.encoder_stream_instructions(payload):
                if kind == "insert_nameref":
                    py.append(info["value"])
                elif kind == "insert_literal":
                    py += [info["name"], info["value"]]
            assert got(lits) == expect(py)
            n_enc += len(lits)
        else:
            rc, lits = qhuff.scan_field_section(payload)
            try:
                py = Q.field_section_literals(payload)
            except Q.Truncated:
                assert rc == qhuff.ETRUNC
                continue
            assert rc == qhuff.OK
            assert got(lits) == expect(py)
            assert all(l.kind in (qhuff.LIT_NAME, qhuff.LIT_VALUE)
                       for l in lits)
            n_sec += len(lits)
    assert n_enc + n_sec > 50


@pytest.mark.parametrize("name", STREAMS)
def test_encoder_stream_resumes_at_any_split(name):
    enc = b"".join(p for sid, p in frames(name) if sid == 0)
    _, whole, used = qhuff.scan_encoder_stream(enc)
    rng = random.Random(5)
    pos, acc = 0, []
    pending = b""
    while pos < len(enc) or pending:
        k = rng.randrange(1, 40)
        chunk = pending + enc[pos:pos + k]
        base = pos - len(pending)
        pos += k
        rc, lits, c = qhuff.scan_encoder_stream(chunk, base)
        assert rc == qhuff.OK
        acc += lits
        pending = chunk[c:]
        if pos >= len(enc):
            break
    assert got(acc) == got(whole)
    assert used + len(pending) == len(enc)


def test_scan_reference_header_block_kats():
    kats = json.load(open(os.path.join(G, "kat_header_blocks.json")))
    for k in kats["header_blocks"]:
        sec = bytes.fromhex(k["prefix"] + k["header"])
        rc, lits = qhuff.scan_field_section(sec)
        assert rc == qhuff.OK, k["source"]
        assert got(lits) == expect(Q.field_section_literals(sec))
        rc, lits, used = qhuff.scan_encoder_stream(bytes.fromhex(k["enc"]))
        assert rc == qhuff.OK and used == len(k["enc"]) // 2


def test_scan_reference_enc_stream_kats():
    kats = json.load(open(os.path.join(G, "kat_enc_stream.json")))
    for k in kats["enc_stream"]:
        buf = bytes.fromhex(k["enc_stream"])
        rc, lits, used = qhuff.scan_encoder_stream(buf)
        assert rc == qhuff.OK, k["source"]
        py = []
        for kind, info in Q.encoder_stream_instructions(buf):
            if kind == "insert_nameref":
                py.append(info["value"])
            elif kind == "insert_literal":
                py += [info["name"], info["value"]]
        assert got(lits) == expect(py)


def test_scan_rejects_like_the_reference():
    # 64-bit overflow in the Required Insert Count (lsqpack_dec_int -> -2)
    assert qhuff.scan_field_section(b"\xff" + b"\xff" * 10 + b"\x01")[0] \
        == qhuff.EPROTO
    # a literal length >= 2^24 (lsqpack_dec_int24 -> -2)
    big = b"\x00\x00" + b"\x51\x7f\x80\x80\x80\x08"
    assert qhuff.scan_field_section(big)[0] == qhuff.EPROTO
    # ends inside a literal / inside the prefix
    assert qhuff.scan_field_section(b"\x00\x00\x5f\x00\x85\xa4\xa9")[0] \
        == qhuff.ETRUNC
    assert qhuff.scan_field_section(b"")[0] == qhuff.ETRUNC
    # an empty field section is a prefix only
    assert qhuff.scan_field_section(b"\x00\x00") == (qhuff.OK, [])
    # encoder stream: a partial instruction is left for the next chunk
    rc, lits, used = qhuff.scan_encoder_stream(b"\xc0\x8b\xf1\xe3")
    assert rc == qhuff.OK and lits == [] and used == 0
    # duplicate index >= 2^24
    assert qhuff.scan_encoder_stream(b"\x1f\xff\xff\xff\x08")[0] \
        == qhuff.EPROTO


# ---- LSXPACK_MAX_STRLEN (lsqpack.c:3682-3685, 3769-3772, 3350-3351) --------

def clamp_kat():
    with open(os.path.join(G, "kat_header_alloc_clamp.json")) as f:
        return json.load(f)


def int_kat():
    with open(os.path.join(G, "kat_int.json")) as f:
        return json.load(f)


def _int_cases():
    kat = int_kat()
    cases = list(kat["dec_int"])
    # (fed whole by the reference test, not byte by byte: its error comes
    # at the 10th continuation byte, before the buffer's end)
    cases.append(dict(kat["overlong_full_buffer"], whole=True))
    return cases


@pytest.mark.parametrize("case", _int_cases(), ids=lambda c: c["source"])
def test_dec_int_reference_vectors(case):
    """test/test_int.c:19-183 (tests[] and test_overlong_integer_full_buffer,
    extracted by make_golden.py): the pre-parse's integer decoder
    (qhuff_frames.cpp dec_int, exported as qhuff_dec_int) returns the
    reference's value for every 0 vector, QHUFF_EPROTO for every -2, and
    QHUFF_ETRUNC for every strict prefix (the reference's -1 loop,
    test_int.c:202-208).  Then each vector is driven through the scanners
    themselves: as a field section's Required Insert Count (8-bit prefix) or
    S + Delta Base (7-bit), and as an encoder-stream Set Dynamic Table
    Capacity (5-bit)."""
    enc = bytes.fromhex(case["encoded"])
    pb, ret = case["prefix_bits"], case["retval"]
    assert ret in (0, -2)
    rc, val, used = qhuff.dec_int(enc, pb)
    if ret == 0:
        assert (rc, val, used) == (qhuff.OK, int(case["decoded"]), len(enc))
        # the Python restatement the fuzz tests use agrees
        assert Q.dec_int(enc, 0, pb) == (int(case["decoded"]), len(enc))
    else:
        assert rc == qhuff.EPROTO
        with pytest.raises(Q.ProtoError):
            Q.dec_int(enc, 0, pb)
    # strict prefixes: -1 from the reference; past 1 + 10 bytes the loop
    # of lsqpack.c:2405-2425 stops reading (M = 70) and decides there
    nfix = min(len(enc), 11) if case.get("whole") else len(enc)
    for k in range(nfix):
        assert qhuff.dec_int(enc[:k], pb)[0] == qhuff.ETRUNC, k
    for k in range(nfix, len(enc)):
        assert qhuff.dec_int(enc[:k], pb)[0] == rc, k
    want = qhuff.OK if ret == 0 else qhuff.EPROTO
    if pb in (7, 8):
        # field section: RIC (8) then delta base (7); the vectors' bits above
        # a 7-bit prefix are 0 (S = 0)
        assert pb == 8 or enc[0] & 0x80 == 0
        wrap = (lambda b: b + b"\x00") if pb == 8 else (lambda b: b"\x00" + b)
        assert qhuff.scan_field_section(wrap(enc))[0] == want
        assert Q.ref_scan_field_section(wrap(enc))[0] == \
            ("ok" if ret == 0 else "proto")
        # (a strict prefix of the RIC is the whole section: a delta-base byte
        # after it would be read as its next continuation byte)
        pre = (lambda b: b) if pb == 8 else wrap
        for k in range(nfix):
            assert qhuff.scan_field_section(pre(enc[:k]))[0] == qhuff.ETRUNC
    if pb == 5:
        # encoder stream: 001xxxxx Set Dynamic Table Capacity (lsqpack_dec_int,
        # no 2^24 limit); a partial instruction is left unconsumed
        assert enc[0] & 0xe0 == 0
        ins = bytes([enc[0] | 0x20]) + enc[1:]
        rc, lits, used = qhuff.scan_encoder_stream(ins)
        assert (rc, lits, used) == ((qhuff.OK, [], len(ins)) if ret == 0
                                    else (qhuff.EPROTO, [], 0))
        for k in range(1, len(ins)):
            assert qhuff.scan_encoder_stream(ins[:k]) == (qhuff.OK, [], 0)


def test_dec_int_args():
    assert qhuff.dec_int(b"\x01", 0)[0] == qhuff.EINVAL
    assert qhuff.dec_int(b"\x01", 9)[0] == qhuff.EINVAL
    # bits above the prefix are ignored
    assert qhuff.dec_int(b"\xea", 5) == (qhuff.OK, 10, 1)


def field_line(first, prefix_bits, payload, huffman=False):
    """one string literal: H bit above an N-bit prefixed length, then the
    payload (RFC 9204 4.5.4 / 4.5.6 shapes)"""
    if huffman:
        first |= 1 << prefix_bits
    return Q.enc_int(first, len(payload), prefix_bits) + payload


def test_alloc_clamp_kats():
    """test/test_header_alloc_clamp.c:108-135: an over-long declared value /
    name length is LQRHS_ERROR right after the length (not 'need more
    bytes': the payload is absent)."""
    kat = clamp_kat()
    assert kat["max_strlen"] == qhuff.MAX_STRLEN == Q.MAX_STRLEN
    assert len(kat["cases"]) == 2
    for case in kat["cases"]:
        assert case["expect"] == "LQRHS_ERROR"
        blk = bytes.fromhex(case["block"])
        assert qhuff.scan_field_section(blk)[0] == qhuff.EPROTO, case["source"]
        assert Q.ref_scan_field_section(blk)[0] == "proto"


@pytest.mark.parametrize("shape", ["nameref", "literal_name", "literal_value",
                                   "postbase"])
@pytest.mark.parametrize("n", [65535, 65536, 70000])
def test_alloc_clamp_present_bytes(shape, n):
    """a literal of n bytes whose payload IS present: accepted up to
    LSXPACK_MAX_STRLEN, rejected (EPROTO) above it -- round 4 returned OK
    for a complete 70,000-byte value."""
    big = b"x" * n
    if shape == "nameref":           # 01NT + 4-bit static index 0
        line = b"\x50" + field_line(0, 7, big)
    elif shape == "literal_name":    # 001NH + 3-bit name length
        line = field_line(0x20, 3, big) + field_line(0, 7, b"v")
    elif shape == "literal_value":
        line = field_line(0x20, 3, b"n") + field_line(0, 7, big)
    else:                            # 0000N + 3-bit post-base index
        line = b"\x00" + field_line(0, 7, big)
    blk = b"\x00\x00" + line
    rc, lits = qhuff.scan_field_section(blk)
    want = qhuff.OK if n <= qhuff.MAX_STRLEN else qhuff.EPROTO
    assert rc == want
    assert Q.ref_scan_field_section(blk)[0] == ("ok" if rc == qhuff.OK
                                                 else "proto")
    if rc == qhuff.OK:
        assert max(l.len for l in lits) == n
    # declared, payload absent: still EPROTO above the limit, ETRUNC below
    rc2 = qhuff.scan_field_section(blk[:-(n // 2)] if shape != "literal_name"
                                   else blk[:8])[0]
    assert rc2 == (qhuff.ETRUNC if n <= qhuff.MAX_STRLEN else qhuff.EPROTO)


def test_encoder_stream_not_clamped():
    """the encoder stream has no LSXPACK_MAX_STRLEN rule (its bound is the
    table capacity, lsqpack.c:4661-4667, which a framing scan does not
    know): a 70,000-byte value is scanned as a literal"""
    ins = field_line(0xc0, 6, b"")[:1] + field_line(0, 7, b"y" * 70000)
    rc, lits, used = qhuff.scan_encoder_stream(ins)
    assert rc == qhuff.OK and used == len(ins) and lits[0].len == 70000


# ---- GPU: all literals of the reference streams in one decode batch ---------

@pytest.fixture(scope="module")
def codec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    c = qhuff.Codec(0)
    yield c
    c.close()


def all_literals():
    """Every complete encoder-stream / field-section literal of the golden
    streams, scanned into one concatenated buffer (pos_base per frame)."""
    buf, lits, truth = b"", [], []
    for name in STREAMS:
        strs = Q.qif_strings(data_file(name + ".qif"))
        for sid, payload in frames(name):
            base = len(buf)
            buf += payload
            if sid == 0:
                rc, ls, _ = qhuff.scan_encoder_stream(payload, base)
            else:
                rc, ls = qhuff.scan_field_section(payload, base)
                if rc == qhuff.ETRUNC:
                    continue
            assert rc == qhuff.OK
            lits += ls
            truth += [strs] * len(ls)
    return buf, lits, truth


@pytest.mark.gpu
def test_gpu_decode_all_stream_literals(codec):
    buf, lits, truth = all_literals()
    outs, status = codec.decode_literals_host(buf, lits)
    assert not status.any()
    n_huff = 0
    for l, o, strs in zip(lits, outs, truth):
        payload = buf[l.pos:l.pos + l.len]
        if l.huffman:
            st, want = O.huff_decode(payload)
            assert st == O.OK
            n_huff += 1
        else:
            want = payload
        assert o == want
        # fb-resp carries two empty values the QIF text does not show as
        # such (interop-encode's QIF reader, not the codec)
        assert o in strs or o == b""
    assert n_huff > 100


@pytest.mark.gpu
def test_gpu_decode_literals_with_errors(codec):
    rng = random.Random(11)
    buf, lits = b"", []
    for i in range(3000):
        s = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40)))
        if i % 3:
            s = O.huffman_enc(s[:30]) if i % 5 else s
        lit = qhuff.Literal(len(buf), len(s), int(i % 3 != 0), 7, 2, 0, 0)
        buf += s
        lits.append(lit)
    outs, status = codec.decode_literals_host(buf, lits)
    for l, o, st in zip(lits, outs, status):
        payload = buf[l.pos:l.pos + l.len]
        if l.huffman:
            ost, want = O.huff_decode(payload)
            assert st == (0 if ost == O.OK else 1)
            assert o == (want if ost == O.OK else b"")
        else:
            assert st == 0 and o == payload


def static_name_len(idx):
    with open(os.path.join(G, "qpack_static_table.json")) as f:
        return len(json.load(f)["static_table"][idx][0])


@pytest.mark.gpu
def test_gpu_decode_clamp(codec):
    """header_out_grow_buf (lsqpack.c:3346-3351): a field line's name and
    value are decoded into ONE header buffer that never grows past
    LSXPACK_MAX_STRLEN (round 5 applied the limit to each
    string alone).  With max_len = MAX_STRLEN: a literal name 'nm' takes 2
    of the 65,535 bytes, so a value of 65,533 decoded bytes fits and 65,535
    or 65,536 do not; a static name reference (lsqpack.c:3620-3642 copies
    the table's name into the buffer) takes its name's length; a dynamic
    reference (table with the reference) leaves the value checked alone.
    Without a limit (encoder-stream use) everything decodes.  The
    reference's over-long declared lengths (test_header_alloc_clamp.c)
    never reach the decode: the scan rejects their blocks."""
    for case in clamp_kat()["cases"]:
        assert qhuff.scan_field_section(bytes.fromhex(case["block"]))[0] \
            == qhuff.EPROTO
    buf, lits, want = b"", [], []
    # (huffman name?, name part, decoded value length, expected statuses)
    nm_h = O.huffman_enc(b"nm")
    cases = [(field_line(0x20, 3, b"nm"), 65533, [0, 0]),
             (field_line(0x20, 3, b"nm"), 65534, [0, 1]),
             (field_line(0x20, 3, b"nm"), 65535, [0, 1]),
             (field_line(0x20, 3, b"nm"), 65536, [0, 1]),
             (field_line(0x20, 3, nm_h, huffman=True), 65533, [0, 0]),
             (field_line(0x20, 3, nm_h, huffman=True), 65534, [0, 1]),
             (field_line(0x20, 3, b"nm"), 10, [0, 0]),
             (field_line(0x20, 3, b"nm"), 0, [0, 0]),
             # static name refs: index 0 (:authority, 10), 2 (age, 3), 31
             # (a two-byte index)
             (b"\x50", 65535 - static_name_len(0), [0]),
             (b"\x50", 65536 - static_name_len(0), [1]),
             (b"\x52", 65535 - static_name_len(2), [0]),
             (b"\x52", 65536 - static_name_len(2), [1]),
             (Q.enc_int(0x50, 31, 4), 65535 - static_name_len(31), [0]),
             (Q.enc_int(0x50, 31, 4), 65536 - static_name_len(31), [1]),
             # dynamic name ref (T = 0) and post-base name ref: value alone
             (b"\x45", 65535, [0]),
             (b"\x45", 65536, [1]),
             (b"\x02", 65535, [0])]
    for head, n, st in cases:
        h = O.huffman_enc(b"a" * n)
        blk = b"\x00\x00" + head + field_line(0, 7, h, huffman=True)
        rc, ls = qhuff.scan_field_section(blk, len(buf))
        assert rc == qhuff.OK and len(ls) == len(st)
        buf += blk
        lits += ls
        want += [(s_, n if (s_ == 0 and l.kind == qhuff.LIT_VALUE) else None)
                 for s_, l in zip(st, ls)]
    outs, status = codec.decode_literals_host(buf, lits, qhuff.MAX_STRLEN)
    assert list(status) == [s_ for s_, _ in want]
    for o, (s_, n), l in zip(outs, want, lits):
        if s_:
            assert o == b""
        elif n is not None:
            assert o == b"a" * n
        else:
            assert o == b"nm"
    outs, status = codec.decode_literals_host(buf, lits)
    assert not status.any()
    # a raw literal above the limit (only reachable through hand-made spans)
    raw = [qhuff.Literal(0, 70000, 0, 7, 2, 0, 0)]
    outs, status = codec.decode_literals_host(b"z" * 70000, raw,
                                              qhuff.MAX_STRLEN)
    assert list(status) == [1] and outs == [b""]


@pytest.mark.gpu
def test_gpu_decode_no_literals(codec):
    outs, status = codec.decode_literals_host(b"", [])
    assert outs == [] and len(status) == 0
