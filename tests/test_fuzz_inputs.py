"""The reference's adversarial decoder inputs through the literal-span
scanners and the GPU literal decode.

Fixtures: fuzz/decode/{a,b,c,d} -- the AFL seed corpora and preambles of
the reference's decoder fuzzing (tests/golden/fuzz_decode.json, copied by
tests/golden/make_golden.py), read with the framing of bin/fuzz-decode.c:
152-202 (preamble: every record; test case: its first record, size clamped)
or, for the interop-decode dir (c), every record.  Plus bit-flipped and
truncated variants of the reference's interop streams.

CPU: qhuff_scan_field_section / qhuff_scan_encoder_stream (host code in
libqhuff.so) equal a strict Python restatement of the reference's framing
and integer rules (tests/qpack_frames.py ref_scan_*, lsqpack.c:2372-2460,
3567-4046, 4574-4960) in return code, literal spans and consumed bytes.
GPU: every literal the scanners yield -- valid, invalid or truncated
Huffman -- decoded in one launch equals the oracle's lsqpack_huff_decode
(status and bytes)."""
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
RC = {"ok": qhuff.OK, "trunc": qhuff.ETRUNC, "proto": qhuff.EPROTO}


def _read(rel):
    with open(os.path.join(G, rel), "rb") as f:
        return f.read()


def fuzz_records():
    """(label, stream id, payload) of every fixture record."""
    man = json.load(open(os.path.join(G, "fuzz_decode.json")))
    out = []
    for d, ent in sorted(man["dirs"].items()):
        if ent["preamble"]:
            for k, (sid, p) in enumerate(Q.fuzz_records(_read(ent["preamble"]))):
                out.append(("%s/preamble#%d" % (d, k), sid, p))
        for c in ent["cases"]:
            data = _read(c["file"])
            if ent["program"] == "fuzz-decode":
                recs = Q.fuzz_records(data, strict=False, single=True)
            else:
                recs = Q.fuzz_records(data, strict=False)
            for k, (sid, p) in enumerate(recs):
                out.append(("%s#%d" % (c["original"], k), sid, p))
    return out


def mutated_records(n=3000, seed=17):
    """Records of the reference's interop streams with bytes flipped,
    replaced or cut (a deterministic havoc over real QPACK wire data)."""
    rng = random.Random(seed)
    base = []
    for name in ("netbsd", "fb-req", "fb-resp"):
        base += list(Q.read_interop(_read("data/%s.out.256.100.1" % name)))
    out = []
    for i in range(n):
        sid, p = base[rng.randrange(len(base))]
        b = bytearray(p)
        for _ in range(rng.randrange(1, 4)):
            if not b:
                break
            op = rng.randrange(4)
            j = rng.randrange(len(b))
            if op == 0:
                b[j] ^= 1 << rng.randrange(8)
            elif op == 1:
                b[j] = rng.choice((0x00, 0x7f, 0x80, 0xff, rng.randrange(256)))
            elif op == 2:
                del b[j:]
            else:
                b[j:j] = bytes(rng.randrange(256)
                               for _ in range(rng.randrange(1, 12)))
        out.append(("mut#%d" % i, sid, bytes(b)))
    return out


def scan(sid, payload, base=0):
    if sid == 0:
        rc, lits, used = qhuff.scan_encoder_stream(payload, base)
        return rc, lits, used
    rc, lits = qhuff.scan_field_section(payload, base)
    return rc, lits, None


def spans(lits):
    return [(l.pos, l.len, l.huffman, l.prefix_bits, l.hdr_len, l.kind,
             l.instr) for l in lits]


def check_record(label, sid, payload):
    rc, lits, used = scan(sid, payload)
    if sid == 0:
        want, wl, wused = Q.ref_scan_encoder_stream(payload)
        assert (rc, used if rc == qhuff.OK else 0) == (RC[want], wused), label
    else:
        want, wl = Q.ref_scan_field_section(payload)
        assert rc == RC[want], label
    if rc == qhuff.OK:
        assert spans(lits) == wl, label
        for l in lits:
            assert l.pos + l.len <= len(payload)
    return rc, lits


def test_fuzz_fixture_manifest():
    man = json.load(open(os.path.join(G, "fuzz_decode.json")))
    assert sorted(man["dirs"]) == ["a", "b", "c", "d"]
    n = sum(len(e["cases"]) for e in man["dirs"].values())
    assert n == 14
    recs = fuzz_records()
    assert any(sid == 0 for _, sid, _ in recs)
    assert any(sid != 0 for _, sid, _ in recs)


def test_scanners_on_reference_fuzz_corpora():
    seen = {qhuff.OK: 0, qhuff.ETRUNC: 0, qhuff.EPROTO: 0}
    n_lits = 0
    for label, sid, payload in fuzz_records():
        rc, lits = check_record(label, sid, payload)
        seen[rc] += 1
        n_lits += len(lits)
    assert seen[qhuff.OK] > 0 and n_lits > 0


def test_scanners_on_mutated_streams():
    seen = {qhuff.OK: 0, qhuff.ETRUNC: 0, qhuff.EPROTO: 0}
    for label, sid, payload in mutated_records():
        rc, _ = check_record(label, sid, payload)
        seen[rc] += 1
    # the havoc reaches every outcome
    assert all(v > 0 for v in seen.values()), seen


def test_scanners_on_random_bytes():
    rng = random.Random(23)
    for i in range(3000):
        p = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 48)))
        check_record("rand#%d" % i, i & 1, p)


def gather_literals():
    """All literals the scanners yield over the fuzz corpora and the mutated
    streams, concatenated into one buffer (pos_base per record)."""
    buf, lits = b"", []
    for label, sid, payload in fuzz_records() + mutated_records(1500, 29):
        base = len(buf)
        rc, ls, _ = scan(sid, payload, base)
        if rc != qhuff.OK or not ls:
            continue
        buf += payload
        lits += ls
    return buf, lits


@pytest.mark.gpu
def test_gpu_decode_fuzz_literals():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    buf, lits = gather_literals()
    assert len(lits) > 500
    c = qhuff.Codec(0)
    try:
        outs, status = c.decode_literals_host(buf, lits)
        assert c.device_error() == 0
    finally:
        c.close()
    n_bad = 0
    for l, o, st in zip(lits, outs, status):
        payload = buf[l.pos:l.pos + l.len]
        if l.huffman:
            ost, want = O.huff_decode(payload)
            assert st == (0 if ost == O.OK else 1), (l.pos, payload.hex())
            assert o == (want if ost == O.OK else b""), (l.pos, payload.hex())
            n_bad += ost != O.OK
        else:
            assert st == 0 and o == payload
    assert n_bad > 0                         # the corpora carry rejects
    assert np.asarray(status).dtype == np.uint8
