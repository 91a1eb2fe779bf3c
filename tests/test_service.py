"""The low-latency service (qhuff_svc_*, qhuff_service.hip) on the GPU against
the CPU oracle: the same bit-exact bar as the batch kernels (output bytes,
out_off, per-string status), on the reference's known-answer vectors,
random batches that take every tile path (staged, unstaged slow path, long
codes, rejects), the slot limits, the host-path fallback, concurrent callers,
the kernel's idle exit and relaunch, and the routing of a context's own
host-path and per-string calls through an attached service."""
import json
import os
import random
import threading
import time

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAX_N, MAX_B = 1024, 65536


@pytest.fixture(scope="module")
def codec():
    import qhuff
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    c = qhuff.Codec(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def svc(codec):
    s = codec.service()
    yield s
    s.close()


def pack(strings, base=0):
    off = np.zeros(len(strings) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strings], out=off[1:])
    data = np.frombuffer(b"\0" * base + b"".join(strings), dtype=np.uint8).copy()
    return data, off + base


def check_enc(svc, data, off, mode):
    out, oo = svc.encode(data, off, mode)
    o_out, o_off = O.encode_batch(data, off, mode)
    assert np.array_equal(oo, o_off)
    assert np.array_equal(out, o_out)
    return out, oo


def check_dec(svc, data, off):
    out, oo, st = svc.decode(data, off)
    o_out, o_off, o_st = O.decode_batch(data, off)
    assert np.array_equal(st, o_st)
    assert np.array_equal(oo, o_off)
    assert np.array_equal(out, o_out)
    return out, oo, st


def rand_strings(rng, n, lo, hi, alphabet=None):
    out = []
    for _ in range(n):
        k = rng.randint(lo, hi)
        if alphabet is None:
            out.append(bytes(rng.getrandbits(8) for _ in range(k)))
        else:
            out.append(bytes(rng.choice(alphabet) for _ in range(k)))
    return out


def test_svc_kats(svc):
    kat = json.load(open(os.path.join(G, "kat_huff_decode.json")))
    ok = [bytes.fromhex(k["huff"]) for k in kat["decode_ok"]]
    bad = [bytes.fromhex(k["huff"]) for k in kat["decode_error"]]
    data, off = pack(ok + bad)
    out, oo, st = check_dec(svc, data, off)
    for i, k in enumerate(kat["decode_ok"]):
        assert st[i] == 0
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["plain"])
    assert list(st[len(ok):]) == [1] * len(bad)
    data, off = pack([bytes.fromhex(k["plain"]) for k in kat["decode_ok"]])
    out, oo = check_enc(svc, data, off, 0)
    for i, k in enumerate(kat["decode_ok"]):
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["huff"])
    es = json.load(open(os.path.join(G, "kat_enc_str.json")))["enc_str"]
    data, off = pack([bytes.fromhex(k["str"]) for k in es])
    out, oo = check_enc(svc, data, off, 3)
    for i, k in enumerate(es):
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["out"])


@pytest.mark.parametrize("n,lo,hi", [(1, 0, 40), (5, 8, 64), (63, 0, 64),
                                     (64, 8, 64), (65, 8, 64), (200, 0, 120),
                                     (300, 100, 200), (1024, 0, 63)])
def test_svc_random_round_trip(svc, n, lo, hi):
    """every encode mode, then the payloads back; byte strings over the whole
    alphabet (codes up to 30 bits), tiles past the 3 KB stage (slow path)"""
    rng = random.Random(n * 1000 + hi)
    tok = list(b"abcdefghijklmnopqrstuvwxyz0123456789-_.:/=")
    for alpha in (None, tok):
        strs = rand_strings(rng, n, lo, hi, alpha)
        if sum(map(len, strs)) > MAX_B:
            strs = strs[:len(strs) // 2]
        data, off = pack(strs, base=rng.randint(0, 9))
        for mode in (0, 3, 5, 7):
            check_enc(svc, data, off, mode)
        enc, eo = check_enc(svc, data, off, 0)
        check_dec(svc, enc, eo)


def test_svc_rejects_and_garbage(svc):
    """random bytes as Huffman input: mostly rejects (status 1, no output),
    some accepted -- exactly as the oracle says"""
    rng = random.Random(7)
    strs = rand_strings(rng, 500, 0, 40)
    data, off = pack(strs)
    _, _, st = check_dec(svc, data, off)
    assert 0 < int(st.sum()) < len(strs)


def test_svc_empty_and_limits(codec, svc):
    served0 = svc.stats()[0]
    # no strings; empty strings
    out, oo = svc.encode(np.zeros(1, np.uint8), np.zeros(1, np.uint32))
    assert list(oo) == [0]
    data, off = pack([b""] * 7)
    check_enc(svc, data, off, 0)
    check_enc(svc, data, off, 7)
    check_dec(svc, data, off)
    # exactly a full slot: 1024 strings, 65536 bytes
    rng = random.Random(3)
    strs = [bytes(rng.getrandbits(8) for _ in range(64)) for _ in range(MAX_N)]
    data, off = pack(strs)
    assert int(off[-1]) == MAX_B
    check_enc(svc, data, off, 5)
    served1, launches, fb0 = svc.stats()
    assert served1 > served0
    # one string over: the context's host path
    data, off = pack(strs + [b"x"])
    check_enc(svc, data, off, 0)
    data, off = pack([b"y" * (MAX_B + 1)])
    check_enc(svc, data, off, 0)
    assert svc.stats()[2] == fb0 + 2


def test_svc_bad_offsets(svc):
    import qhuff
    data = np.zeros(16, np.uint8)
    with pytest.raises(qhuff.QhuffError):
        svc.encode(data, np.array([0, 5, 3], dtype=np.uint32))


def test_svc_concurrent_callers(svc):
    """8 threads x 60 calls, each a different batch (more callers than a
    few slots are free at a time): every result bit-exact"""
    served0 = svc.stats()[0]
    errors = []

    def worker(t):
        try:
            rng = random.Random(100 + t)
            for i in range(60):
                strs = rand_strings(rng, rng.randint(1, 80), 0, 50)
                data, off = pack(strs)
                if i % 2:
                    check_enc(svc, data, off, (0, 3, 5, 7)[i % 4])
                else:
                    enc, eo = O.encode_batch(data, off, 0)
                    check_dec(svc, enc, eo)
        except Exception as e:                      # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors[:3]
    assert svc.stats()[0] - served0 == 8 * 60


def test_svc_idle_exit_and_relaunch():
    """a service whose kernel leaves after 2 ms idle is started again by the
    next call, which a pending request survives"""
    import qhuff
    c = qhuff.Codec(0)
    try:
        s = c.service(idle_us=2000)
        data, off = pack([b"www.example.com", b"no-cache"])
        check_enc(s, data, off, 0)
        launches0 = s.stats()[1]
        for _ in range(3):
            time.sleep(0.05)
            check_enc(s, data, off, 7)
        assert s.stats()[1] >= launches0 + 3
        s.close()
        s2 = c.service()                            # close + reopen
        check_enc(s2, data, off, 3)
        s2.close()
    finally:
        c.close()


def test_svc_routes_context_host_calls(codec, svc):
    """with a service attached, the context's host-path batch calls and the
    per-string mirrors that fit a slot are served by it"""
    served0 = svc.stats()[0]
    data, off = pack([b"custom-key", b"custom-value", b""])
    out, oo = codec.encode_host(data, off, 0)
    o_out, o_off = O.encode_batch(data, off, 0)
    assert np.array_equal(oo, o_off) and np.array_equal(out, o_out)
    d_out, d_oo, st = codec.decode_host(out, oo)
    assert bytes(d_out) == b"custom-keycustom-value" and not st.any()
    for p in (3, 5, 7):
        assert codec.enc_enc_str(p, b"www.example.com") == \
            O.enc_enc_str(p, b"www.example.com")
    st, dst, n_src = codec.huff_decode(O.huffman_enc(b"text/html"))[:3]
    assert st == 0 and dst == b"text/html"
    assert svc.stats()[0] >= served0 + 6


def test_svc_shared_context_for_lsqpack_shims(codec, svc):
    """qhuff_lsqpack_set_context: the reference-signature per-string calls of
    several threads on one context with the service attached"""
    import qhuff
    L = qhuff.lib()
    served0 = svc.stats()[0]
    assert L.qhuff_lsqpack_set_context(codec._ctx) == qhuff.OK
    errors = []

    def worker(t):
        try:
            rng = random.Random(t)
            for _ in range(40):
                s = bytes(rng.choice(b"abcdefgh-./:0123") for _ in
                          range(rng.randint(0, 60)))
                assert qhuff.lsqpack_enc_enc_str(5, s) == O.enc_enc_str(5, s)
                h = O.huffman_enc(s)
                st, dst = qhuff.lsqpack_huff_decode(h, len(s) + 1)[:2]
                assert st == 0 and dst == s
        except Exception as e:                      # noqa: BLE001
            errors.append(repr(e))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
    finally:
        L.qhuff_lsqpack_set_context(None)
    assert not errors, errors[:3]
    assert svc.stats()[0] >= served0 + 4 * 40 * 2


@pytest.mark.parametrize("size", [3073, 20000, 65536])
def test_svc_single_long_string(svc, size):
    """one string longer than the 3 KB stage: the service's scratch path
    (input copied to the slot's device scratch, the tile loop, results
    copied back) -- valid strings in every mode and back, and invalid
    Huffman input of the same sizes"""
    rng = random.Random(size)
    tok = list(b"abcdefghijklmnopqrstuvwxyz0123456789-_.:/=")
    s = bytes(rng.choice(tok) for _ in range(size))
    data, off = pack([s], base=rng.randint(0, 5))
    served0, _, fb0 = svc.stats()
    for mode in (0, 3, 5, 7):
        check_enc(svc, data, off, mode)
    enc, eo = check_enc(svc, data, off, 0)
    assert int(eo[-1]) <= MAX_B                     # the payload fits a slot
    check_dec(svc, enc, eo)
    # invalid: the payload with its last byte's padding broken, and random
    # bytes (EOS or bad padding somewhere)
    bad = enc.copy()
    bad[int(eo[-1]) - 1] &= 0x7f
    _, _, st = check_dec(svc, bad, eo)
    junk = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(size)),
                         dtype=np.uint8).copy()
    check_dec(svc, junk, np.array([0, size], dtype=np.uint32))
    served1, _, fb1 = svc.stats()
    assert fb1 == fb0 and served1 >= served0 + 8   # none took the host path


def test_svc_shared_context_long_strings_threaded(codec, svc):
    """calls too large for a slot (> 64 KB) on a shared context
    go through the service's fallback lock, so threads mixing them with
    small calls still get bit-exact results"""
    import qhuff
    L = qhuff.lib()
    assert L.qhuff_lsqpack_set_context(codec._ctx) == qhuff.OK
    errors = []

    def worker(t):
        try:
            rng = random.Random(50 + t)
            for i in range(6):
                k = MAX_B + 1 + rng.randint(0, 5000) if i % 2 else \
                    rng.randint(0, 200)
                s = bytes(rng.choice(b"abcdefgh-./:0123") for _ in range(k))
                want = O.enc_enc_str(7, s)
                assert qhuff.lsqpack_enc_enc_str(7, s, dst_len=len(want) + 8) \
                    == want
                h = O.huffman_enc(s)
                st, dst = qhuff.lsqpack_huff_decode(h, len(s) + 1)[:2]
                assert st == 0 and dst == s
        except Exception as e:                      # noqa: BLE001
            errors.append(repr(e))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
    finally:
        L.qhuff_lsqpack_set_context(None)
    assert not errors, errors[:3]


def test_set_context_requires_service():
    """a context without a service cannot be shared (its host path is not
    thread-safe): QHUFF_EINVAL, and the default contexts stay in use"""
    import qhuff
    c = qhuff.Codec(0)
    try:
        L = qhuff.lib()
        assert L.qhuff_lsqpack_set_context(c._ctx) == qhuff.EINVAL
        assert qhuff.lsqpack_enc_enc_str(5, b"dude") == O.enc_enc_str(5, b"dude")
    finally:
        c.close()
