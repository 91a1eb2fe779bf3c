"""Exact-signature shims (include/qhuff_lsqpack.h) against the oracle.

qhuff_lsqpack_huff_decode has lsqpack_huff_decode's argument list
(lsqpack.c:3520-3535): a complete string is decoded on the GPU; when dst is
too small the shim returns what the reference's huff_decode_fast returns
(END_DST with n_dst/n_src backed off to a byte boundary,
lsqpack.c:5438-5450), or, where the reference falls into its nibble decoder
(slow_path, lsqpack.c:5452-5465), hands the rest to the registered streaming
decoder -- for invalid strings as well (END_DST where dst runs out before the
error, qhuff_fastwalk.h fast_walk_invalid).  Here the registered decoder is the oracle's restatement of
lsqpack_huff_decode_full, so every (status, n_dst, n_src, dst) must equal
the oracle's oq_huff_decode on the same arguments, for every dst_len.

qhuff_lsqpack_enc_enc_str has lsqpack_enc_enc_str's argument list
(lsqpack.c:839-876) and is compared the same way, including the -1 result
for every too-small dst_len and the kept high bits of dst[0].
"""
import ctypes as C
import json
import os
import random

import pytest

import _paths  # noqa: F401
import oracle_lib as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# byte classes by code length: 5-8 bit, 10-15 bit, >16 bit (slow path)
SHORT = b"0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJ-./:=_ %"
MID = b"!\"#$&'()*+,;<>?@[\\]^`{|}~"
LONG = bytes(range(0, 32)) + bytes(range(128, 256))


def _oracle_full_ptr():
    return C.cast(O.lib().oq_huff_decode_full, C.c_void_p).value


@pytest.fixture
def shim():
    import qhuff
    qhuff.lib().qhuff_lsqpack_set_decode_full(_oracle_full_ptr())
    yield qhuff
    qhuff.lib().qhuff_lsqpack_set_decode_full(None)


def oracle_decode(src, dst_len, state=None, final=1):
    s = C.create_string_buffer(bytes(src), len(src) + 1)
    d = C.create_string_buffer(max(dst_len, 1))
    st = state if state is not None else O.DecState(0, 0, 0)
    rv = O.lib().oq_huff_decode(s, len(src), d, dst_len, C.byref(st), final)
    return rv.status, d.raw[:rv.n_dst], rv.n_dst, rv.n_src


def shim_decode(qhuff, src, dst_len, state=None, final=1):
    st = None
    if state is not None:
        st = qhuff.DecodeState(state.resume, state.state, state.eos)
    status, out, n_dst, n_src, _ = qhuff.lsqpack_huff_decode(
        src, dst_len, st, final)
    return status, out, n_dst, n_src


def _strings(seed, n, alpha, lo, hi):
    rng = random.Random(seed)
    return [bytes(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))
            for _ in range(n)]


def _every_dst_len(qhuff, enc):
    n = len(O.huff_decode(enc)[1])
    for dst_len in range(0, n + 2):
        got = shim_decode(qhuff, enc, dst_len)
        want = oracle_decode(enc, dst_len)
        assert got == want, (enc.hex(), dst_len, got, want)


@pytest.mark.gpu
def test_decode_kats_every_dst_len(shim):
    kat = json.load(open(os.path.join(GOLD, "kat_huff_decode.json")))
    for k in kat["decode_ok"]:
        _every_dst_len(shim, bytes.fromhex(k["huff"]))
    for k in kat["decode_error"]:
        src = bytes.fromhex(k["huff"])
        got = shim_decode(shim, src, 4 * len(src) + 8)
        assert got == oracle_decode(src, 4 * len(src) + 8) and got[0] == O.ERROR


@pytest.mark.gpu
@pytest.mark.parametrize("alpha,lo,hi,n", [
    (SHORT, 0, 40, 60),                 # fast loop + last-window paths
    (SHORT + MID, 1, 40, 60),           # 10-15 bit codes: 1-2 per window
    (SHORT + MID + LONG, 1, 24, 60),    # >16 bit codes: slow_path hand-off
    (LONG, 1, 8, 40),
])
def test_decode_random_every_dst_len(shim, alpha, lo, hi, n):
    for s in _strings(len(alpha) * 100 + hi, n, alpha, lo, hi):
        enc = O.huffman_enc(s)
        assert O.huff_decode(enc)[1] == s
        _every_dst_len(shim, enc)


@pytest.mark.gpu
def test_decode_invalid_strings(shim):
    """Random bytes: valid ones decode exactly; invalid ones as the
    reference reports them when dst is ample (ERROR, with the nibble
    decoder's n_dst / n_src where a long code sent the reference there)."""
    rng = random.Random(7)
    for _ in range(300):
        src = bytes(rng.randrange(256) for _ in range(rng.randint(1, 12)))
        cap = 4 * len(src) + 8
        assert shim_decode(shim, src, cap) == oracle_decode(src, cap)


@pytest.mark.gpu
def test_decode_invalid_every_dst_len(shim):
    """an invalid complete string at every dst_len --
    the EOS code after short and long codes, padding of 8+ ones, padding
    that is not all ones, random bytes, the reference's must-reject KATs --
    gives oq_huff_decode's (status, dst, n_dst, n_src): END_DST where dst
    runs out before the reference reaches the error, the nibble decoder's
    result where a long code sends it there, else ERROR (the GPU's Keep
    kernel returns the bytes before the error; qhuff_fastwalk.h
    fast_walk_invalid replays the reference over them)."""
    import test_fastwalk as TF
    kat = json.load(open(os.path.join(GOLD, "kat_huff_decode.json")))
    inputs = [bytes.fromhex(k["huff"]) for k in kat["decode_error"]]
    inputs += TF._invalid_inputs(33)[:150]
    n_end_dst = 0
    for enc in inputs:
        for dst_len in range(0, 8 * len(enc) // 5 + 3):
            got = shim_decode(shim, enc, dst_len)
            want = oracle_decode(enc, dst_len)
            assert got == want, (enc.hex(), dst_len, got, want)
            n_end_dst += want[0] == O.END_DST
    assert n_end_dst > 100


@pytest.mark.gpu
def test_decode_end_dst_caller_loop(shim):
    """The reference decoder's own loop on END_DST (lsqpack.c:3713-3742:
    keep the state, continue from n_src with a grown dst, final while input
    remains) gives the same step sequence through the shim as through the
    oracle, and rebuilds the string."""
    for s in _strings(11, 40, SHORT + MID + LONG, 4, 40):
        enc = O.huffman_enc(s)
        runs = []
        for dec, st in ((lambda *a: shim.lsqpack_huff_decode(*a)[:4],
                         shim.DecodeState(0, 0, 0)),
                        (oracle_decode, O.DecState(0, 0, 0))):
            out, pos, dst_len, steps = b"", 0, 3, []
            while True:
                status, part, n_dst, n_src = dec(enc[pos:], dst_len, st, 1)
                steps.append((status, n_dst, n_src))
                assert status in (O.OK, O.END_DST), steps
                out += part
                pos += n_src
                if status == O.OK:
                    break
                dst_len += 3
            assert out == s
            runs.append(steps)
        assert runs[0] == runs[1]


@pytest.mark.gpu
def test_decode_streaming_goes_to_registered_decoder(shim):
    """resume != 0 or final == 0 is the reference's streaming decoder."""
    s = b"www.example.com/some/path?query=value"
    enc = O.huffman_enc(s)
    a = O.DecState(0, 0, 0)
    b = O.DecState(0, 0, 0)
    got1 = shim_decode(shim, enc[:5], 64, a, final=0)
    want1 = oracle_decode(enc[:5], 64, b, final=0)
    assert got1 == want1 and want1[0] == O.END_SRC


@pytest.mark.gpu
def test_decode_without_registered_decoder():
    """No streaming decoder: streaming input is ERROR; a slow-path stop is
    the byte-boundary END_DST (a prefix of the string)."""
    import qhuff
    qhuff.lib().qhuff_lsqpack_set_decode_full(None)
    enc = O.huffman_enc(b"ab")
    assert shim_decode(qhuff, enc, 8, O.DecState(0, 0, 0), final=0)[0] \
        == O.ERROR
    for s in _strings(5, 30, SHORT + LONG, 2, 20):
        enc = O.huffman_enc(s)
        for dst_len in range(len(s)):
            st, part, n_dst, n_src = shim_decode(qhuff, enc, dst_len)
            assert st == O.END_DST and n_dst <= dst_len
            assert part == s[:n_dst] and n_src <= len(enc)
        assert shim_decode(qhuff, enc, len(s))[:2] == (O.OK, s)


@pytest.mark.gpu
@pytest.mark.parametrize("prefix", [3, 5, 7])
def test_enc_enc_str_every_dst_len(prefix):
    import qhuff
    kat = json.load(open(os.path.join(GOLD, "kat_enc_str.json")))["enc_str"]
    strs = [bytes.fromhex(k["str"]) for k in kat]
    strs += _strings(3, 30, SHORT + MID, 0, 40)
    strs += _strings(4, 20, LONG, 0, 30)          # raw (Huffman not shorter)
    strs.append(bytes(200))                       # multi-byte length prefix
    for i, s in enumerate(strs):
        first = (0xff << (prefix + 1)) & 0xff if i % 2 else 0
        need = len(O.enc_enc_str(prefix, s, first))
        for dst_len in sorted({0, 1, need - 1, need, need + 5}
                              | set(range(0, min(need + 1, 12)))):
            if dst_len < 0:
                continue
            got = qhuff.lsqpack_enc_enc_str(prefix, s, first, dst_len)
            want = O.enc_enc_str(prefix, s, first, dst_len)
            assert got == want, (prefix, s.hex(), dst_len, got, want)
