"""Pin the CPU oracle to the reference's own known answers and to the
reference-encoded QPACK streams (tests/golden/, made by make_golden.py)."""
import json
import os

import pytest

import oracle_lib as O
import qpack_frames as Q

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


def test_code_table_kats():
    # RFC 7541 Appendix B: 'a' = 00011 (5 bits), EOS = 30 ones
    assert O.code_of(ord("a")) == (0x3, 5)
    assert O.code_of(256) == (0x3FFFFFFF, 30)
    from fractions import Fraction
    kraft = sum(Fraction(1, 2 ** O.code_of(s)[1]) for s in range(257))
    assert kraft == 1


DEC = load("kat_huff_decode.json")


@pytest.mark.parametrize("kat", DEC["decode_ok"], ids=lambda k: k["source"])
@pytest.mark.parametrize("full", [False, True])
def test_decode_kats(kat, full):
    huff, plain = bytes.fromhex(kat["huff"]), bytes.fromhex(kat["plain"])
    st, out = O.huff_decode(huff, full=full)
    assert st == O.OK and out == plain


@pytest.mark.parametrize("kat", DEC["decode_ok"], ids=lambda k: k["source"])
def test_encode_reproduces_decode_kats(kat):
    huff, plain = bytes.fromhex(kat["huff"]), bytes.fromhex(kat["plain"])
    assert O.huffman_enc(plain) == huff
    assert O.enc_str_size(plain) == len(huff)


@pytest.mark.parametrize("kat", DEC["decode_ok"], ids=lambda k: k["source"])
def test_decode_kats_chunked(kat):
    """test/test_huff_dec.c:318-371: every (in chunk, out chunk) pair through
    the resumable decoder.  The 2,807-byte case is 'expensive' in the
    reference (-e); here it runs a strided subset of the pairs."""
    huff, plain = bytes.fromhex(kat["huff"]), bytes.fromhex(kat["plain"])
    if len(huff) * len(plain) < 150000:
        ins, outs = range(1, len(huff) + 1), range(1, len(plain) + 1)
    else:
        ins = list(range(1, 9)) + list(range(9, len(huff) + 1, 397))
        outs = list(range(1, 9)) + list(range(9, len(plain) + 1, 331))
    for ic in ins:
        for oc in outs:
            st, out = O.huff_decode_chunked(huff, ic, oc)
            assert st == O.OK and out == plain, (ic, oc)


@pytest.mark.parametrize("kat", DEC["decode_error"], ids=lambda k: k["source"])
@pytest.mark.parametrize("full", [False, True])
def test_bad_padding_rejected(kat, full):
    st, _ = O.huff_decode(bytes.fromhex(kat["huff"]), full=full)
    assert st == O.ERROR


@pytest.mark.parametrize("kat", load("kat_enc_str.json")["enc_str"],
                         ids=lambda k: k["source"])
def test_enc_str_kats(kat):
    r = O.enc_enc_str(kat["prefix_bits"], bytes.fromhex(kat["str"]),
                      dst_len=0x1000)
    assert r == bytes.fromhex(kat["out"])
    assert len(r) == kat["retval"]


def test_enc_str_dst_too_small():
    # lsqpack.c:849-859 / 862-872: -1 when dst_len cannot hold the literal
    assert O.enc_enc_str(3, b"aaa", dst_len=2) == -1
    assert O.enc_enc_str(3, b"aaa", dst_len=3) == bytes.fromhex("0a18c7")
    assert O.enc_enc_str(7, b"\x80\x90", dst_len=2) == -1


def test_enc_str_preserves_high_bits():
    # lsqpack.c:852-853: bits above prefix+1 of dst[0] are kept
    r = O.enc_enc_str(5, b"www.netbsd.org", first_byte=0xC0)
    assert r[0] & 0xC0 == 0xC0 and r[0] & 0x20 == 0x20


STATIC = [(n.encode("latin-1"), v.encode("latin-1"))
          for n, v in load("qpack_static_table.json")["static_table"]]


def decode_literal(lit):
    if lit["huffman"]:
        st, out = O.huff_decode(lit["payload"])
        assert st == O.OK
        return out
    return lit["payload"]


@pytest.mark.parametrize("kat", load("kat_enc_stream.json")["enc_stream"],
                         ids=lambda k: k["source"])
def test_encoder_stream_kats(kat):
    """test/test_read_enc_stream.c: encoder-stream bytes -> dynamic table."""
    table = []
    for kind, info in Q.encoder_stream_instructions(
            bytes.fromhex(kat["enc_stream"])):
        if kind == "insert_nameref":
            name = (STATIC[info["index"]][0] if info["static"]
                    else table[-1 - info["index"]][0])
            table.append((name, decode_literal(info["value"])))
        elif kind == "insert_literal":
            table.append((decode_literal(info["name"]),
                          decode_literal(info["value"])))
        elif kind == "dup":
            table.append(table[-1 - info["index"]])
        elif kind == "capacity" and info["capacity"] == 0:
            table = []
    want = [(bytes.fromhex(n), bytes.fromhex(v)) for n, v in kat["dyn_table"]]
    assert table == want


def check_literals_reencode(lits):
    """Every literal the reference wrote must be reproduced bit-exactly by
    lsqpack_enc_enc_str on its decoded string (H choice, prefixed length,
    Huffman bytes and the preserved instruction bits)."""
    for lit in lits:
        s = decode_literal(lit)
        hib = lit["first_byte"] & ~((1 << (lit["prefix_bits"] + 1)) - 1) & 0xFF
        again = O.enc_enc_str(lit["prefix_bits"], s, first_byte=hib)
        assert again == lit["wire"], (lit, s)
        if lit["huffman"]:
            assert O.huffman_enc(s) == lit["payload"]
    return [decode_literal(l) for l in lits]


@pytest.mark.parametrize("kat", load("kat_header_blocks.json")["header_blocks"],
                         ids=lambda k: k["source"])
def test_header_block_kats(kat):
    """test/test_qpack.c header_block_tests[]: every literal in the expected
    encoder stream and header block re-encodes bit-exactly and decodes to one
    of the test's header names/values."""
    strings = set()
    for n, v in kat["headers"]:
        strings |= {bytes.fromhex(n), bytes.fromhex(v)}
    lits = []
    for kind, info in Q.encoder_stream_instructions(bytes.fromhex(kat["enc"])):
        if kind == "insert_nameref":
            lits.append(info["value"])
        elif kind == "insert_literal":
            lits += [info["name"], info["value"]]
    lits += Q.field_section_literals(bytes.fromhex(kat["prefix"] + kat["header"]))
    for s in check_literals_reencode(lits):
        assert s in strings


@pytest.mark.parametrize("corpus", ["netbsd", "fb-req", "fb-resp"])
def test_reference_encoded_streams(corpus):
    """fuzz/input/256.100.1/<corpus>.out.256.100.1 were written by the
    reference's interop-encode (-t 256 -s 100 -a 1) from test/qifs/<corpus>.qif.
    Every Huffman and raw literal in them decodes to a QIF name/value and
    re-encodes bit-exactly."""
    data = open(os.path.join(G, "data", corpus + ".out.256.100.1"), "rb").read()
    qif = open(os.path.join(G, "data", corpus + ".qif"), "rb").read()
    lits = Q.stream_literals(data)
    assert len(lits) > 20
    n_huff = sum(l["huffman"] for l in lits)
    assert n_huff > 10
    # b"": the reference's encoder also inserts name-only dynamic entries
    # (empty value) into the encoder stream
    strings = Q.qif_strings(qif) | {b""}
    for s in check_literals_reencode(lits):
        assert s in strings


def test_oracle_self_consistency_random():
    """Fast (16-bit window) and full (nibble FSM) decoders agree on random
    valid and random garbage inputs, and encode->decode round-trips."""
    import random
    rng = random.Random(7)
    for i in range(3000):
        n = rng.randrange(0, 80)
        alpha = [bytes(range(256)), b"abcdefghijklmnopqrstuvwxyz0123456789-_./",
                 b"\x01\x02\x06\x5c\x8d" + b"abc"][i % 3]
        s = bytes(rng.choice(alpha) for _ in range(n))
        h = O.huffman_enc(s)
        assert O.huff_decode(h) == (O.OK, s)
        assert O.huff_decode(h, full=True) == (O.OK, s)
        g = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 24)))
        a, b = O.huff_decode(g), O.huff_decode(g, full=True)
        assert a == b, g.hex()
