"""Exhaustive and constructed-adversarial parity (SURVEY.md 8(c) fixture
plan items (ii) and (iii), 8(d) config 3's 1 % invalid variant and
alphabet C at full size).

* every single byte and every byte pair (65,792 strings) in every encode
  mode, and decoded back;
* decode inputs built bit by bit to hit each reject clause of the D3 rule
  (lsqpack.c:5362-5426, 3482-3497): the EOS code embedded at a symbol
  boundary, >= 8 padding bits, non-ones padding, long codes cut short;
  the oracle's fast (huff_decode_fast, lsqpack.c:5234) and full
  (lsqpack_huff_decode_full, lsqpack.c:3443) restatements must agree on
  them before the GPU is compared (CPU tests), then the GPU must match
  status and bytes (gpu tests);
* the 1M-string config-3 batch with every 100th payload corrupted, and the
  1M-string long-code alphabet C (token alphabet + ~2 % of {1,2,6,92,141}).
"""
import random

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O

TOKEN = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
LONG = bytes([1, 2, 6, 92, 141])
EOS_BITS = "1" * 30


def pack(strings):
    off = np.zeros(len(strings) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strings], out=off[1:])
    data = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    return data, off


def bits_of(s: bytes) -> str:
    out = []
    for b in s:
        c, n = O.code_of(b)
        out.append(format(c, "0%db" % n))
    return "".join(out)


def to_bytes(bits: str) -> bytes:
    assert len(bits) % 8 == 0
    return int(bits, 2).to_bytes(len(bits) // 8, "big") if bits else b""


def pad_ones(bits: str) -> str:
    return bits + "1" * (-len(bits) % 8)


def all_pairs():
    return [bytes([a]) for a in range(256)] + \
        [bytes([a, b]) for a in range(256) for b in range(256)]


def invalid_cases(seed=3, n=400):
    """(category, payload) pairs; every payload violates one D3 clause."""
    rng = random.Random(seed)
    cases = []
    for _ in range(n):
        pre = bytes(rng.choice(TOKEN + LONG) for _ in range(rng.randint(0, 12)))
        suf = bytes(rng.choice(TOKEN) for _ in range(rng.randint(0, 12)))
        bp = bits_of(pre)
        # (a) EOS at a symbol boundary, anything after it
        cases.append(("eos", to_bytes(pad_ones(bp + EOS_BITS + bits_of(suf)))))
        # (b) 8..15 bits of (all-ones) padding after the last symbol
        k = rng.randint(8, 15)
        cases.append(("pad8", to_bytes(pad_ones(bp + "1" * k))))
        # (c) 1..7 padding bits that are not all ones: 1^(r-1) 0 is no code
        # of <= 7 bits (5-bit codes start with 0, 6-bit codes end at 101101,
        # 7-bit codes at 1111011) and only a prefix of longer ones
        r = -len(bp) % 8
        if r:
            cases.append(("pad0", to_bytes(bp + "1" * (r - 1) + "0")))
    return cases


def truncated_long_codes(seed=4, n=300):
    """Strings ending in a long code (14..30 bits) cut after k bits, then
    padded with ones: rejected or not as the D3 rule says (a cut of <= 7
    leading ones is plain padding); only parity is asserted."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        pre = bytes(rng.choice(TOKEN) for _ in range(rng.randint(0, 10)))
        sym = rng.choice(LONG + bytes(range(200, 256)))
        c = bits_of(bytes([sym]))
        k = rng.randint(1, len(c) - 1)
        out.append(to_bytes(pad_ones(bits_of(pre) + c[:k])))
    return out


# ---- CPU: the oracle agrees with itself on the constructed inputs ----------

def test_oracle_rejects_constructed_invalid():
    cases = invalid_cases()
    assert {c for c, _ in cases} == {"eos", "pad8", "pad0"}
    for cat, h in cases:
        assert O.huff_decode(h)[0] == O.ERROR, (cat, h.hex())
        assert O.huff_decode(h, full=True)[0] == O.ERROR, (cat, h.hex())


def test_oracle_fast_full_agree_on_truncations_and_pairs():
    trunc = truncated_long_codes()
    data, off = pack(trunc)
    fo, foo, fst = O.decode_batch(data, off)
    uo, uoo, ust = O.decode_batch(data, off, full=True)
    assert np.array_equal(fst, ust) and np.array_equal(fo, uo)
    assert fst.sum() > len(trunc) // 2 and (fst == 0).sum() > 0
    # every pair round-trips through the oracle
    strs = all_pairs()
    data, off = pack(strs)
    h, ho = O.encode_batch(data, off, 0)
    d, do, st = O.decode_batch(h, ho)
    assert not st.any() and np.array_equal(d, data)


# ---- GPU ----------------------------------------------------------------------

@pytest.fixture(scope="module")
def codec():
    torch = pytest.importorskip("torch")
    import qhuff
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    c = qhuff.Codec(0)
    yield c
    c.close()


def _enc(codec, data, off, mode):
    import torch
    d = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if len(data):
        d[:len(data)] = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).to(torch.int32).cuda()
    out, oo = codec.encode(d, o, mode)
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    oo = oo.cpu().numpy().view(np.uint32)
    return out[:int(oo[-1])].cpu().numpy(), oo


def _dec(codec, data, off):
    import torch
    d = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if len(data):
        d[:len(data)] = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64)).to(torch.int32).cuda()
    out, oo, st = codec.decode(d, o)
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    oo = oo.cpu().numpy().view(np.uint32)
    return out[:int(oo[-1])].cpu().numpy(), oo, st.cpu().numpy()


def _check_dec(codec, data, off):
    g = _dec(codec, data, off)
    o = O.decode_batch(data, off)
    assert np.array_equal(g[2], o[2]), "status differs"
    assert np.array_equal(g[1], o[1]), "out_off differs"
    assert np.array_equal(g[0], o[0]), "bytes differ"
    return g


@pytest.mark.gpu
def test_gpu_all_bytes_and_pairs(codec):
    strs = all_pairs()
    rng = random.Random(1)
    rng.shuffle(strs)                # mix code lengths inside every tile
    data, off = pack(strs)
    for mode in (0, 3, 5, 7):
        g, go = _enc(codec, data, off, mode)
        o, oo = O.encode_batch(data, off, mode)
        assert np.array_equal(go, oo) and np.array_equal(g, o), mode
    h, ho = O.encode_batch(data, off, 0)
    out, oo, st = _check_dec(codec, h, ho)
    assert not st.any() and np.array_equal(out, data)


@pytest.mark.gpu
def test_gpu_constructed_invalid(codec):
    cases = invalid_cases()
    valid = [O.huffman_enc(bytes(random.Random(i).choice(TOKEN)
                                 for _ in range(i % 40))) for i in range(400)]
    trunc = truncated_long_codes()
    strs = [h for _, h in cases] + valid + trunc
    idx = list(range(len(strs)))
    random.Random(2).shuffle(idx)    # invalid strings spread over the tiles
    data, off = pack([strs[i] for i in idx])
    out, oo, st = _check_dec(codec, data, off)
    pos = {j: k for k, j in enumerate(idx)}
    for j in range(len(cases)):
        assert st[pos[j]] == 1, cases[j][0]
    for j in range(len(cases), len(cases) + len(valid)):
        assert st[pos[j]] == 0


@pytest.mark.gpu
def test_gpu_config3_one_percent_invalid(codec):
    """Config 3 at full size with every 100th payload followed by a 0xff
    byte (>= 8 bits of padding, always rejected): status and bytes equal
    the oracle's; 10,486 rejects."""
    import qhuff
    data, off = qhuff.synth_batch(1 << 20)
    h, ho = O.encode_batch(data, off, 0)
    strs = [bytes(h[ho[i]:ho[i + 1]]) for i in range(len(ho) - 1)]
    for i in range(0, len(strs), 100):
        strs[i] += b"\xff"
    d2, o2 = pack(strs)
    out, oo, st = _check_dec(codec, d2, o2)
    assert int(st.sum()) == len(range(0, len(strs), 100))


@pytest.mark.gpu
def test_gpu_config2_alphabet_c_full_size(codec):
    """Alphabet C: token alphabet with ~2 % long-code bytes,
    1M strings: every encode mode equals the oracle, decode round-trips."""
    import qhuff
    alpha = TOKEN * 5 + LONG                      # 5 / 230 = 2.2 %
    data, off = qhuff.synth_batch(1 << 20, seed=7, alphabet=alpha)
    frac = np.isin(data, np.frombuffer(LONG, np.uint8)).mean()
    assert 0.015 < frac < 0.03
    for mode in (0, 7):
        g, go = _enc(codec, data, off, mode)
        o, oo = O.encode_batch(data, off, mode)
        assert np.array_equal(go, oo) and np.array_equal(g, o), mode
        if mode == 0:
            h, ho = g, go
    out, oo, st = _check_dec(codec, h, ho)
    assert not st.any() and np.array_equal(out, data)
