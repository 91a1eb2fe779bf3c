"""The wave-cooperative long-string decode (qhuff_decode_impl.h coop_decode),
restated segment for segment in Python and checked against the oracle on
the reference's own header corpora (tests/golden/data/*.qif) and on
adversarial strings.  CPU only: this pins the algorithm -- segment sizes,
guessed walks with marks (A), walks on to the meeting points (B), the
round loop, the per-segment counts and the exact first symbol starts of the
write walks (W) -- independently of the kernel; the GPU parity tests
(test_gpu_parity.py test_decode_cooperative_*) pin the kernel itself.

The model's walks decode symbol by symbol; the kernel's decode one or two a
step and cut a step's second symbol at the walk's limit, which gives the
same symbol starts."""
import os
import random

import pytest

import _paths  # noqa: F401
import oracle_lib as O

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
SEG_MIN = 64                                 # kSegMin (bits)


def _codes():
    by_len = {}
    for s in range(257):
        c, n = O.code_of(s)
        by_len.setdefault(n, {})[c] = s
    return by_len


BY_LEN = _codes()


def _walker(h):
    """symbol at bit p of h (followed by 8 zero bytes, as the next strings'
    bytes in the stage): (sym, len)"""
    data = h + b"\x00" * 8
    nb = len(data) * 8
    v = int.from_bytes(data, "big")

    def at(p):
        w = (v >> (nb - p - 30)) & ((1 << 30) - 1)
        for L in range(5, 31):
            s = BY_LEN.get(L, {}).get(w >> (30 - L))
            if s is not None:
                return s, L
        return None, 31
    return at


def seg_bits(hls):
    """S for a tile whose cooperative strings have these Huffman lengths:
    the kernel's sum_j max(1, bits_j / S) <= 64 choice"""
    tot = 8 * sum(hls)
    dv = 64 - len(hls)
    return max(SEG_MIN, (((tot + dv - 1) // dv) + 31) & ~31)


def coop_model(h, S=None):
    """(output bytes, rounds) of coop_decode for the Huffman string h (alone
    in its tile unless S is given), or None where the kernel falls back to
    the one-lane decode."""
    at = _walker(h)
    b1 = nbits = 8 * len(h)
    if S is None:
        S = seg_bits([len(h)])
    hv = int.from_bytes(h, "big")

    def pad_bad(pos):
        """the D3 rule on the bits [pos, b1) after the last symbol"""
        r = b1 - pos
        return r >= 8 or (hv & ((1 << r) - 1)) != (1 << r) - 1
    nseg = max(1, nbits // S)
    assert nseg <= 64
    s = [k * S for k in range(nseg)]
    stop = [(k + 1) * S if k + 1 < nseg else b1 for k in range(nseg)]
    marks = set()

    def walk(pos, lim, mode, out=None):
        """symbols starting in [pos, lim) that end inside the string (the
        rest is padding), an EOS or overrun ends the walk; Check stops on a
        marked start"""
        n = 0
        while pos < lim:
            if mode == "check" and pos in marks:
                return pos, n, True, False
            sym, L = at(pos)
            if sym is None or pos + L > b1:
                return pos, n, False, pad_bad(pos)
            if sym == 256:
                return pos, n, False, True
            if mode == "mark":
                marks.add(pos)
            if out is not None:
                out.append(sym)
            n += 1
            pos += L
        return pos, n, False, False

    # A
    E, C = [], []
    for k in range(nseg):
        e, c, _, _ = walk(s[k], stop[k], "mark")
        E.append(e)
        C.append(c)
    # B, rounds
    cs = list(E)
    X, K, met = [0] * nseg, [0] * nseg, [False] * nseg
    redo = [k + 1 < nseg for k in range(nseg)]
    rounds = 0
    while any(redo):
        rounds += 1
        assert rounds <= 64
        for k in range(nseg):
            if redo[k]:
                X[k], K[k], met[k], _ = walk(cs[k], stop[k + 1], "check")
        for k in range(nseg - 1):
            tE = X[k - 1] if k >= 1 and not met[k - 1] else E[k]
            redo[k] = tE != cs[k]
            cs[k] = tE
        redo[nseg - 1] = False
    T = [C[0]] + [K[k - 1] + (sum(1 for q in marks if X[k - 1] <= q < stop[k])
                              if met[k - 1] else 0) for k in range(1, nseg)]
    if sum(T) > (8 * len(h)) // 5:
        return None
    # W
    out = []
    for k in range(nseg):
        o = []
        x, m, _, bad = walk(0 if k == 0 else cs[k - 1], stop[k], "emit", o)
        if bad or m != T[k] or (k + 1 < nseg and x != cs[k]):
            return None
        if k + 1 == nseg and b1 - x >= 8:
            return None                      # padding of 8 bits or more
        out += o
    return bytes(out), rounds


def corpus_strings():
    out = []
    for q in ("fb-req.qif", "fb-resp.qif", "long-codes.qif", "netbsd.qif"):
        with open(os.path.join(G, q), "rb") as f:
            for line in f.read().split(b"\n"):
                if line and not line.startswith(b"#"):
                    n, _, v = line.partition(b"\t")
                    out += [n, v]
    return out


def test_coop_model_corpus():
    """Every distinct corpus string of more than 40 Huffman bytes (the
    kernel's threshold is 128; shorter ones exercise one- and two-segment
    walks): the cooperative result is the decoded string."""
    rounds = []
    long = {s for s in corpus_strings() if len(O.huffman_enc(s)) > 40}
    assert len(long) > 100
    for s in sorted(long):
        r = coop_model(O.huffman_enc(s))
        assert r is not None and r[0] == s
        rounds.append(r[1])
    assert max(rounds) < 16


def test_coop_model_tiles():
    """Several cooperative strings of one tile share the lanes: S from all
    of them, every string decoded right, never more than 64 segments."""
    rng = random.Random(3)
    long = sorted({s for s in corpus_strings() if len(O.huffman_enc(s)) > 128})
    for _ in range(40):
        k = rng.randint(1, 6)
        strs = rng.sample(long, k)
        hs = [O.huffman_enc(x) for x in strs]
        S = seg_bits([len(h) for h in hs])
        assert sum(max(1, 8 * len(h) // S) for h in hs) <= 64
        for x, h in zip(strs, hs):
            r = coop_model(h, S)
            assert r is not None and r[0] == x


@pytest.mark.parametrize("alpha", [b"abcdefghijklmnopqrstuvwxyz0123456789-_./",
                                   bytes(range(256)),
                                   b"\x01\x02\x06\x5c\x8dabcdefgh"])
def test_coop_model_random(alpha):
    rng = random.Random(len(alpha))
    for n in (130, 161, 257, 600, 1461, 3000):
        s = bytes(rng.choice(alpha) for _ in range(n))
        h = O.huffman_enc(s)
        if len(h) <= 128:
            continue
        r = coop_model(h)
        assert r is not None and r[0] == s


def test_coop_model_invalid_falls_back():
    """Corrupted long strings (an EOS code spliced in, bit flips, a cut, 8
    padding bits, padding that is not all ones): whenever the oracle rejects
    a string the model hands it back to the one-lane decode (None); what it
    does return is the oracle's output."""
    rng = random.Random(7)
    cases = []
    for i in range(60):
        s = bytes(rng.choice(b"abcdefghijklmnop/=;") for _ in range(
            rng.randint(200, 900)))
        h = bytearray(O.huffman_enc(s))
        k = i % 5
        if k == 0:
            # EOS on a symbol boundary: after the codes of a prefix
            j = rng.randrange(1, len(s))
            bits = sum(O.code_of(c)[1] for c in s[:j])
            v = int.from_bytes(bytes(h), "big")
            nb = 8 * len(h)
            hi, lo = v >> (nb - bits), v & ((1 << (nb - bits)) - 1)
            v2 = (((hi << 30) | 0x3fffffff) << (nb - bits)) | lo
            h = bytearray(v2.to_bytes((nb + 30 + 7) // 8 + 1, "big"))
        elif k == 1:
            at = rng.randrange(len(h))
            h[at] ^= 1 << rng.randrange(8)
        elif k == 2:
            h = h[:-rng.randint(1, 3)]
        elif k == 3:
            h += b"\xff"
        else:
            npad = 8 * len(h) - sum(O.code_of(c)[1] for c in s)
            if npad:
                h[-1] &= 0xff ^ (1 << (npad - 1))
        cases.append(bytes(h))
    rejected = 0
    for h in cases:
        st, out = O.huff_decode(h)
        r = coop_model(h)
        if st != O.OK:
            rejected += 1
            assert r is None
        elif r is not None:
            assert r[0] == out
    assert rejected > 30
