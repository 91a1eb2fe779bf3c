"""GPU parity: the HIP path through the C-ABI (libqhuff.so) against the CPU
oracle and the reference's own golden vectors.  Bit-exact everywhere (this
is byte/integer work): output bytes, out_off, and per-string status."""
import json
import os
import random

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O
import qpack_frames as Q

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def codec():
    import qhuff
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    c = qhuff.Codec(0)
    yield c
    c.close()


def pack(strings):
    off = np.zeros(len(strings) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strings], out=off[1:])
    data = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    return data, off


def to_dev(data, off, pad_front=0):
    """Device copies; pad_front shifts the data pointer off 16-byte alignment
    and in_off[0] away from 0 (both allowed by the ABI)."""
    d = torch.zeros(len(data) + pad_front + 16, dtype=torch.uint8,
                    device="cuda")
    if len(data):
        d[pad_front:pad_front + len(data)] = torch.from_numpy(data).cuda()
    o = torch.from_numpy(off.astype(np.int64) + pad_front).to(torch.int32).cuda()
    return d, o


def gpu_encode(codec, data, off, mode=0, pad_front=0):
    d, o = to_dev(data, off, pad_front)
    out, out_off = codec.encode(d, o, mode)
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    oo = out_off.cpu().numpy().view(np.uint32)
    return out[:int(oo[-1])].cpu().numpy(), oo


def gpu_decode(codec, data, off, pad_front=0):
    d, o = to_dev(data, off, pad_front)
    out, out_off, status = codec.decode(d, o)
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    oo = out_off.cpu().numpy().view(np.uint32)
    return out[:int(oo[-1])].cpu().numpy(), oo, status.cpu().numpy()


def check_encode(codec, data, off, mode, pad_front=0):
    g_out, g_off = gpu_encode(codec, data, off, mode, pad_front)
    o_out, o_off = O.encode_batch(data, off, mode)
    assert np.array_equal(g_off, o_off)
    assert np.array_equal(g_out, o_out)
    return g_out, g_off


def check_decode(codec, data, off, pad_front=0):
    g_out, g_off, g_st = gpu_decode(codec, data, off, pad_front)
    o_out, o_off, o_st = O.decode_batch(data, off)
    assert np.array_equal(g_st, o_st)
    assert np.array_equal(g_off, o_off)
    assert np.array_equal(g_out, o_out)
    return g_out, g_off, g_st


def load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)


# ---- golden vectors ------------------------------------------------------------

def test_decode_kats(codec):
    kat = load("kat_huff_decode.json")
    ok = [bytes.fromhex(k["huff"]) for k in kat["decode_ok"]]
    bad = [bytes.fromhex(k["huff"]) for k in kat["decode_error"]]
    data, off = pack(ok + bad)
    out, oo, st = gpu_decode(codec, data, off)
    for i, k in enumerate(kat["decode_ok"]):
        assert st[i] == 0
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["plain"])
    assert list(st[len(ok):]) == [1] * len(bad)
    check_decode(codec, data, off)


def test_encode_kats(codec):
    kat = load("kat_huff_decode.json")["decode_ok"]
    data, off = pack([bytes.fromhex(k["plain"]) for k in kat])
    out, oo = check_encode(codec, data, off, 0)
    for i, k in enumerate(kat):
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["huff"])


def test_enc_str_kats(codec):
    kat = load("kat_enc_str.json")["enc_str"]
    assert all(k["prefix_bits"] == 3 for k in kat)
    data, off = pack([bytes.fromhex(k["str"]) for k in kat])
    out, oo = check_encode(codec, data, off, 3)
    for i, k in enumerate(kat):
        assert bytes(out[oo[i]:oo[i + 1]]) == bytes.fromhex(k["out"])
        assert oo[i + 1] - oo[i] == k["retval"]


@pytest.mark.parametrize("corpus", ["netbsd", "fb-req", "fb-resp"])
def test_reference_encoded_stream_literals(codec, corpus):
    """Every literal of the reference-encoded interop stream: the GPU decodes
    the Huffman payloads, and re-encodes the strings with the same framing
    bit for bit (prefix 3/5/7 batches)."""
    raw = open(os.path.join(G, "data", corpus + ".out.256.100.1"), "rb").read()
    lits = Q.stream_literals(raw)
    huff = [l for l in lits if l["huffman"]]
    data, off = pack([l["payload"] for l in huff])
    out, oo, st = check_decode(codec, data, off)
    assert not st.any()
    plain = {id(l): bytes(out[oo[i]:oo[i + 1]]) for i, l in enumerate(huff)}
    for p in (3, 5, 7):
        sel = [l for l in lits if l["prefix_bits"] == p]
        if not sel:
            continue
        strs = [plain[id(l)] if l["huffman"] else l["payload"] for l in sel]
        d2, o2 = pack(strs)
        e, eo = check_encode(codec, d2, o2, p)
        for i, l in enumerate(sel):
            wire = bytearray(e[eo[i]:eo[i + 1]])
            hib = l["first_byte"] & ~((1 << (p + 1)) - 1) & 0xFF
            wire[0] |= hib
            assert bytes(wire) == l["wire"]


def test_qif_corpus_round_trip(codec):
    """All names and values of the four QIF corpora (real header strings,
    incl. long-codes.qif): encode in every mode, decode the payloads."""
    strs = []
    for fn in ("netbsd.qif", "fb-req.qif", "fb-resp.qif", "long-codes.qif"):
        for hl in Q.qif_header_lists(open(os.path.join(G, "data", fn), "rb").read()):
            for n, v in hl:
                strs += [n, v]
    data, off = pack(strs)
    for mode in (0, 3, 5, 7):
        check_encode(codec, data, off, mode)
    h, ho = check_encode(codec, data, off, 0)
    out, oo, st = check_decode(codec, h, ho)
    assert not st.any()
    assert np.array_equal(out, data) and np.array_equal(oo, off - off[0])


# ---- synthetic + adversarial batches -----------------------------------------------

def rand_strings(rng, n, alpha, lo, hi):
    return [bytes(rng.choice(alpha) for _ in range(rng.randint(lo, hi)))
            for _ in range(n)]


ALPHAS = {
    "token": b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, ",
    "all": bytes(range(256)),
    "long": b"\x01\x02\x06\x5c\x8d" + b"abcdefgh",
    "high": bytes(range(128, 256)),
}


@pytest.mark.parametrize("alpha", sorted(ALPHAS))
@pytest.mark.parametrize("mode", [0, 3, 5, 7])
def test_encode_random(codec, alpha, mode):
    rng = random.Random(hash((alpha, mode)) & 0xffff)
    strs = rand_strings(rng, 3000, ALPHAS[alpha], 0, 80)
    data, off = pack(strs)
    check_encode(codec, data, off, mode)
    check_encode(codec, data, off, mode, pad_front=5)


@pytest.mark.parametrize("alpha", sorted(ALPHAS))
def test_decode_random_valid(codec, alpha):
    rng = random.Random(len(alpha))
    strs = rand_strings(rng, 3000, ALPHAS[alpha], 0, 80)
    data, off = pack(strs)
    h, ho = O.encode_batch(data, off, 0)
    out, oo, st = check_decode(codec, h, ho)
    assert not st.any() and np.array_equal(out, data)
    check_decode(codec, h, ho, pad_front=3)


def test_decode_garbage(codec):
    """Random bytes: mostly rejects (EOS, long padding, non-ones padding);
    accept/reject and output must match the reference decoder exactly."""
    rng = random.Random(11)
    strs = [bytes(rng.randrange(256) for _ in range(rng.randint(0, 40)))
            for _ in range(20000)]
    # near-valid: valid encodings with the last byte perturbed / extended
    for i in range(5000):
        s = rand_strings(rng, 1, ALPHAS["token"], 1, 30)[0]
        h = bytearray(O.huffman_enc(s))
        r = i % 4
        if r == 0:
            h[-1] ^= 1 << rng.randrange(8)
        elif r == 1:
            h += b"\xff"
        elif r == 2:
            h += bytes([rng.randrange(256)])
        else:
            h = h[:-1]
        strs.append(bytes(h))
    # EOS and long ones runs embedded
    strs += [b"\xff\xff\xff\xfc", b"\xff\xff\xff\xff", b"\x00\xff\xff\xff\xff",
             b"\xfe\xff\xff\xff\xff\x80", b"\x1f\xff", b"\x1f\xff\xff",
             b"\x7f", b"\x3f", b"\x0f\xff"]
    data, off = pack(strs)
    out, oo, st = check_decode(codec, data, off)
    assert st.sum() > 1000 and (st == 0).sum() > 1000


@pytest.mark.parametrize("lo,hi", [(30, 90), (100, 400), (0, 2000)])
def test_multi_unit_tiles(codec, lo, hi):
    """Tiles whose input overflows the LDS stage are coded as several units
    by one workgroup (and single strings past the stage read from global):
    every mode, both directions, mixed with ordinary tiles."""
    rng = random.Random(lo * 7 + hi)
    strs = (rand_strings(rng, 3000, ALPHAS["token"], lo, hi)
            + rand_strings(rng, 2000, ALPHAS["token"], 8, 64)
            + rand_strings(rng, 1000, ALPHAS["long"], lo, hi))
    rng.shuffle(strs)
    data, off = pack(strs)
    for mode in (0, 7):
        check_encode(codec, data, off, mode)
    h, ho = O.encode_batch(data, off, 0)
    out, oo, st = check_decode(codec, h, ho)
    assert not st.any() and np.array_equal(out, data)
    assert codec.device_error() == 0


def test_big_tile_slots(codec):
    """Tiles past the stages whose output fits a big-tile slot (12 KB,
    qhuff_pipeline.h): one string of 3.2-5 KB among short ones (input past
    the stage: the string walked in global memory into the slot), runs of
    ~1 KB strings (several staged units), and tiles just over the stage;
    mixed with ordinary tiles so big tiles sit among pending ones."""
    rng = random.Random(77)
    strs = []
    for t in range(60):
        k = t % 3
        if k == 0:
            tile = (rand_strings(rng, 63, ALPHAS["token"], 0, 20)
                    + rand_strings(rng, 1, ALPHAS["token"], 3200, 5000))
        elif k == 1:
            tile = rand_strings(rng, 8, ALPHAS["all"], 600, 1100) \
                + rand_strings(rng, 56, ALPHAS["token"], 0, 30)
        else:
            tile = rand_strings(rng, 64, ALPHAS["token"], 40, 70)
        rng.shuffle(tile)
        strs += tile
        strs += rand_strings(rng, 64 * 3, ALPHAS["token"], 8, 40)
    data, off = pack(strs)
    for mode in (0, 5, 7):
        check_encode(codec, data, off, mode)
    h, ho = O.encode_batch(data, off, 0)
    out, oo, st = check_decode(codec, h, ho)
    assert not st.any() and np.array_equal(out, data)
    # and invalid strings inside big tiles (statuses and sizes as the oracle)
    h2 = h.copy()
    for i in range(5, len(ho) - 1, 41):
        if ho[i + 1] > ho[i]:
            h2[ho[i + 1] - 1] ^= 0x33
    check_decode(codec, h2, ho)


def test_edge_batches(codec):
    # n = 0
    for mode in (0, 7):
        out, oo = gpu_encode(codec, np.zeros(0, np.uint8),
                             np.zeros(1, np.uint32), mode)
        assert list(oo) == [0]
    # all-empty strings, single string, one huge string (direct paths)
    check_encode(codec, *pack([b""] * 1000), 0)
    check_encode(codec, *pack([b""] * 1000), 7)
    check_decode(codec, *pack([b""] * 1000))
    rng = random.Random(5)
    big = bytes(rng.choice(ALPHAS["all"]) for _ in range(70000))
    for strs in ([b"x"], [big], [b"ab"] * 300 + [big] + [b"cd"] * 300):
        data, off = pack(strs)
        for mode in (0, 3, 7):
            check_encode(codec, data, off, mode)
        h, ho = O.encode_batch(data, off, 0)
        out, oo, st = check_decode(codec, h, ho)
        assert np.array_equal(out, data)
    # strings whose decode output overflows the LDS slot (96 B) and tiles whose
    # input overflows the LDS stage
    strs = rand_strings(rng, 600, ALPHAS["token"], 90, 300)
    data, off = pack(strs)
    check_encode(codec, data, off, 0)
    h, ho = O.encode_batch(data, off, 0)
    check_decode(codec, h, ho)


def _long_tiles(rng, n_tiles, lens, alpha, corrupt=None):
    """Tiles of one long Huffman string (raw length from lens) among 63
    short ones (qhuff_decode_impl.h coop_decode); corrupt(i, h) may alter
    the long string's encoding."""
    strs = []
    for t in range(n_tiles):
        short = [O.huffman_enc(s) for s in
                 rand_strings(rng, 63, ALPHAS["token"], 0, 24)]
        s = bytes(rng.choice(alpha) for _ in range(lens[t % len(lens)]))
        h = O.huffman_enc(s)
        if corrupt is not None:
            h = corrupt(t, bytearray(h))
        pos = rng.randrange(64)
        strs += short[:pos] + [bytes(h)] + short[pos:]
    return pack(strs)


@pytest.mark.parametrize("alpha", ["token", "all", "long"])
def test_decode_cooperative_long_strings(codec, alpha):
    """Strings above the cooperative threshold (128 Huffman bytes) are
    decoded by the whole wave (segment walks, meeting points, counts, then
    the write walk): lengths around the threshold and the segment sizes, up
    to the stage's whole span, each in a tile of short strings; bit-exact
    against the oracle."""
    rng = random.Random(len(alpha) * 31)
    lens = [150, 160, 161, 170, 200, 256, 300, 480, 700, 1000, 1461, 1900, 2400]
    if alpha == "all":
        lens = [80, 81, 100, 130, 200, 400, 700, 900]   # ~2.6x expansion
    data, off = _long_tiles(rng, 3 * len(lens), lens, ALPHAS[alpha])
    out, oo, st = check_decode(codec, data, off)
    assert not st.any()
    check_decode(codec, data, off, pad_front=7)


def test_decode_cooperative_many_per_tile(codec):
    """Tiles holding 2-12 cooperative strings of 130-900 Huffman bytes
    (several strings share the 64 lanes; S from their total, down to the
    64-bit segment minimum) in random places among short ones, a few of
    them invalid; statuses and bytes against the oracle."""
    rng = random.Random(777)
    strs = []
    for t in range(48):
        k = rng.randrange(2, 13)
        longs = set(rng.sample(range(64), k))
        for i in range(64):
            if i in longs:
                s = bytes(rng.choice(ALPHAS["token"])
                          for _ in range(rng.randrange(175, 1200)))
                h = bytearray(O.huffman_enc(s))
                if rng.random() < 0.08:                  # an invalid one
                    h[rng.randrange(len(h))] ^= 1 << rng.randrange(8)
                strs.append(bytes(h))
            else:
                strs.append(O.huffman_enc(
                    bytes(rng.choice(ALPHAS["token"])
                          for _ in range(rng.randrange(0, 40)))))
    data, off = pack(strs)
    out, oo, st = check_decode(codec, data, off)
    assert (st == 0).sum() > 2900


def test_decode_cooperative_invalid(codec):
    """Invalid long strings (an EOS code inside, a flipped bit, non-ones or
    over-long padding, a cut string) take the one-lane decode again: status
    and bytes as the reference decoder."""
    rng = random.Random(4242)

    def corrupt(i, h):
        k = i % 6
        if k == 0:                                   # EOS at a byte boundary
            at = rng.randrange(len(h) // 4, len(h) // 2)
            h[at:at] = b"\xff\xff\xff\xfc"
        elif k == 1:
            at = rng.randrange(len(h))
            h[at] ^= 1 << rng.randrange(8)
        elif k == 2:
            h[-1] &= 0xfe                            # non-ones padding (often)
        elif k == 3:
            h += b"\xff"                             # padding of >= 8 bits
        elif k == 4:
            h = h[:-3]                               # cut
        return h

    data, off = _long_tiles(rng, 120, [200, 500, 1200], ALPHAS["token"],
                            corrupt)
    out, oo, st = check_decode(codec, data, off)
    assert st.sum() > 20 and (st == 0).sum() > 1000


@pytest.mark.parametrize("kernels", ["lean", "full", "auto"])
def test_kernel_variants(kernels):
    """Each kernel of a kind is exact on its own (qhuff_host.cpp pick_full,
    QHUFF_KERNELS): the lean one, which codes big tiles and long strings on
    the round-3 path, the full one (big-tile slots, cooperative long
    strings), and the switch between them -- auto starts lean, and its later
    launches of the same batches run full once the rare flag is set -- on
    big tiles, multi-unit tiles, a tile whose output exceeds a slot (the
    70 KB string among short ones: parked pending tiles, then the slow
    tile) and cooperative strings; each case twice."""
    import qhuff
    old = os.environ.get("QHUFF_KERNELS")
    os.environ["QHUFF_KERNELS"] = kernels
    try:
        c = qhuff.Codec(0)
    finally:
        if old is None:
            del os.environ["QHUFF_KERNELS"]
        else:
            os.environ["QHUFF_KERNELS"] = old
    try:
        rng = random.Random(9)
        huge = bytes(rng.choice(ALPHAS["all"]) for _ in range(70000))
        mixed = pack(rand_strings(rng, 300, ALPHAS["token"], 0, 40) + [huge]
                     + rand_strings(rng, 300, ALPHAS["token"], 0, 40))
        for _ in range(2):
            test_big_tile_slots(c)
            test_multi_unit_tiles(c, 100, 400)
            test_decode_cooperative_long_strings(c, "token")
            test_decode_cooperative_many_per_tile(c)
            test_decode_cooperative_invalid(c)
            for mode in (0, 7):
                check_encode(c, *mixed, mode)
            h, ho = O.encode_batch(*mixed, 0)
            out, oo, st = check_decode(c, h, ho)
            assert np.array_equal(out, mixed[0])
        assert c.device_error() == 0
    finally:
        c.close()


def test_kernel_variant_switch():
    """QHUFF_KERNELS=auto (qhuff_host.cpp pick_full), device-pointer calls:
    without a hint both kinds run their full kernel on every batch -- token
    batches and big-tile batches alike, so a long-string batch's first
    launch after token batches is no slower than its later ones (round 6:
    the round-5 decode history, lean until a launch reported such tiles,
    is gone).  A hint picks the lean kernel for the
    next launch of its kind only (also when that launch is the
    keep-rejected replay).  Outputs checked against the oracle throughout."""
    import qhuff
    if os.environ.get("QHUFF_KERNELS"):
        pytest.skip("QHUFF_KERNELS pins the variant")
    rng = random.Random(11)
    big = []
    for t in range(40):
        tile = rand_strings(rng, 63, ALPHAS["token"], 0, 20) \
            + rand_strings(rng, 1, ALPHAS["token"], 3200, 5000)
        big += tile
    bdata, boff = pack(big)
    bh, bho = O.encode_batch(bdata, boff, 0)
    sdata, soff = qhuff.synth_batch(1 << 14, seed=3)
    sh, sho = O.encode_batch(sdata, soff, 0)
    c = qhuff.Codec(0)
    try:
        E, D = qhuff.KIND_ENCODE, qhuff.KIND_DECODE
        for data, off, h, ho in [(sdata, soff, sh, sho)] * 3 \
                + [(bdata, boff, bh, bho), (sdata, soff, sh, sho)]:
            check_encode(c, data, off, 0)
            check_decode(c, h, ho)
            assert (c.kernel_variant(E), c.kernel_variant(D)) == (1, 1)
        c.batch_hint(E, 0)                       # a hint picks lean, once
        c.batch_hint(D, 0)
        check_encode(c, sdata, soff, 0)
        check_decode(c, sh, sho)
        assert (c.kernel_variant(E), c.kernel_variant(D)) == (0, 0)
        check_encode(c, sdata, soff, 0)
        check_decode(c, sh, sho)
        assert (c.kernel_variant(E), c.kernel_variant(D)) == (1, 1)
        # a hint is consumed by the next launch of its kind whatever that
        # launch is (here the per-string call's own, and its keep-rejected
        # replay): it does not carry over to a later batch launch
        c.batch_hint(D, 0)
        bad = O.huffman_enc(b"abc")[:-1] + b"\x00"
        c.huff_decode(bad)
        check_decode(c, sh, sho)
        assert c.kernel_variant(D) == 1
        assert c.device_error() == 0
    finally:
        c.close()


def test_host_path_variant_from_batch():
    """Host-memory calls choose the kernel variant from the batch itself
    (qhuff_host.cpp host_hint: the offsets are on the host): after 10 token
    batches a batch with big tiles runs the full kernel on its first
    launch, and the next token batch the lean one again -- no history, no
    first-launch cliff (VERDICT r04 item 2 for the paths that can see their
    offsets; device-pointer calls keep pick_full).  Outputs vs the oracle."""
    import qhuff
    if os.environ.get("QHUFF_KERNELS"):
        pytest.skip("QHUFF_KERNELS pins the variant")
    rng = random.Random(12)
    big = []
    for t in range(30):
        big += rand_strings(rng, 62, ALPHAS["token"], 0, 20) \
            + rand_strings(rng, 2, ALPHAS["token"], 150, 3500)
    bdata, boff = pack(big)
    sdata, soff = qhuff.synth_batch(1 << 13, seed=4)
    c = qhuff.Codec(0)
    try:
        E, D = qhuff.KIND_ENCODE, qhuff.KIND_DECODE
        for data, off, want in [(sdata, soff, 0)] * 10 + [(bdata, boff, 1),
                                                         (sdata, soff, 0)]:
            o_out, o_off = O.encode_batch(data, off, 0)
            g_out, g_off = c.encode_host(data, off, 0)
            assert np.array_equal(g_off, o_off)
            assert np.array_equal(g_out[:o_off[-1]], o_out[:o_off[-1]])
            h = o_out[:o_off[-1]].copy()
            d_out, d_off, d_st = c.decode_host(h, o_off)
            assert not d_st.any() and np.array_equal(d_off, off)
            assert np.array_equal(d_out[:off[-1]], data)
            assert (c.kernel_variant(E), c.kernel_variant(D)) == (want, want)
        assert c.device_error() == 0
    finally:
        c.close()


def test_device_batch_hint():
    """qhuff_batch_hint on the device-pointer calls: with the hint computed
    from the caller's host copy of the offsets (qhuff_batch_needs_full) a
    big-tile batch runs the full kernel on its first launch after token
    launches, and a hinted token batch the lean one; outputs exact."""
    import qhuff
    if os.environ.get("QHUFF_KERNELS"):
        pytest.skip("QHUFF_KERNELS pins the variant")
    rng = random.Random(13)
    big = []
    for t in range(30):
        big += rand_strings(rng, 63, ALPHAS["token"], 0, 20) \
            + rand_strings(rng, 1, ALPHAS["token"], 3200, 5000)
    bdata, boff = pack(big)
    sdata, soff = qhuff.synth_batch(1 << 14, seed=3)
    c = qhuff.Codec(0)
    try:
        E = qhuff.KIND_ENCODE
        for _ in range(8):
            c.batch_hint(E, qhuff.batch_needs_full(soff))
            check_encode(c, sdata, soff, 0)
            assert c.kernel_variant(E) == 0
        c.batch_hint(E, qhuff.batch_needs_full(boff))
        check_encode(c, bdata, boff, 0)
        assert c.kernel_variant(E) == 1
        c.batch_hint(E, qhuff.batch_needs_full(soff))
        check_encode(c, sdata, soff, 0)
        assert c.kernel_variant(E) == 0
    finally:
        c.close()


def test_small_grid_long_runs():
    """A grid of a few workgroups (QHUFF_GRID_PCT=4: ~10 of 256) over 4,096
    tiles: each wave codes ~34 tiles, so the ticket claims two iterations
    ahead, the youngest waves' claim stop and the pending-tile ring run
    through many rounds (qhuff_pipeline.h tile_pipeline)."""
    import qhuff
    old = os.environ.get("QHUFF_GRID_PCT")
    os.environ["QHUFF_GRID_PCT"] = "4"
    try:
        c = qhuff.Codec(0)
    finally:
        if old is None:
            del os.environ["QHUFF_GRID_PCT"]
        else:
            os.environ["QHUFF_GRID_PCT"] = old
    try:
        data, off = qhuff.synth_batch(1 << 18, seed=21)
        g_out, g_off = check_encode(c, data, off, 0)
        out, oo, st = check_decode(c, g_out, g_off)
        assert not st.any() and np.array_equal(out, data)
        assert c.device_error() == 0
    finally:
        c.close()


def test_launch_timing(codec):
    """qhuff_timing_enable / qhuff_timing_read (ABIs 4-5): every launch, or
    every k-th of each kind, comes back with its kind and a positive device
    time; the outputs are the same either way."""
    import qhuff
    data, off = qhuff.synth_batch(1 << 14, seed=5)
    codec.timing(True)
    check_encode(codec, data, off, 0)
    check_encode(codec, data, off, 0)
    t = codec.timing_read()
    assert [k for k, _ in t] == [qhuff.KIND_ENCODE] * 2
    assert all(u > 0 for _, u in t)
    codec.timing(True, every=3)
    h, ho = O.encode_batch(data, off, 0)
    for _ in range(7):
        check_encode(codec, data, off, 0)
        check_decode(codec, h, ho)
    t = codec.timing_read()
    codec.timing(False)
    assert [k for k, _ in t].count(qhuff.KIND_ENCODE) == 3      # 0, 3, 6
    assert [k for k, _ in t].count(qhuff.KIND_DECODE) == 3
    assert all(u > 0 for _, u in t)
    check_encode(codec, data, off, 0)
    assert codec.timing_read() == []
    # the per-string entry point on an invalid string: its decode launch is
    # timed, the replay that follows (a decode launch of the keep kernel) is
    # not and leaves the ring alone (it took a slot whose events
    # it never recorded)
    codec.timing(True)
    check_encode(codec, data, off, 0)
    r = codec.huff_decode(b"\xff\xff\xff\xff", 64)
    assert r[0] == qhuff.HUFF_DEC_ERROR
    check_decode(codec, h, ho)
    t = codec.timing_read()
    codec.timing(False)
    E, D = qhuff.KIND_ENCODE, qhuff.KIND_DECODE
    assert [k for k, _ in t] == [E, D, D]
    assert all(u > 0 for _, u in t)


def _launch_shape_check(c, n, seed):
    import qhuff
    data, off = qhuff.synth_batch(n, seed=seed)
    g_out, g_off = check_encode(c, data, off, 0)
    out, oo, st = check_decode(c, g_out, g_off)
    assert not st.any()
    assert np.array_equal(out, data) and np.array_equal(oo, off)


def test_launch_shapes(codec):
    """Batch sizes around the launch-shape boundaries (qhuff_host.cpp
    grid_for): spread launches (one tile per wave, one workgroup per tile up
    to the grid: 1..W tiles) and ticket-group launches with two and three
    prologue tickets per wave (W = the resident grid's waves).  (The
    one-ticket ticket-group launch and its QHUFF_NO_SPREAD switch are gone:
    VERDICT r03 item 6.)"""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    W = n_cu * 12
    tiles = sorted({1, 7, 8, 9, n_cu - 1, n_cu, n_cu + 1, 4 * n_cu + 3,
                    W - 1, W, W + 1, 2 * W, 2 * W + 1, 3 * W, 3 * W + 1})
    for i, t in enumerate(tiles):
        for n in (64 * t, 64 * t - 37):
            if n > 0:
                _launch_shape_check(codec, n, seed=100 + 2 * i + (n % 2))


def test_full_size_round_trip(codec):
    """BASELINE config 2/3 size (1M strings, U[8,64] token alphabet): GPU
    sizes and bytes equal the oracle's; decode(encode(x)) == x."""
    import qhuff
    data, off = qhuff.synth_batch(1 << 20)
    g_out, g_off = check_encode(codec, data, off, 0)
    out, oo, st = check_decode(codec, g_out, g_off)
    assert not st.any()
    assert np.array_equal(out, data) and np.array_equal(oo, off)
    check_encode(codec, data, off, 7)


def test_host_path_and_mirrors(codec):
    rng = random.Random(9)
    strs = rand_strings(rng, 500, ALPHAS["all"], 0, 50)
    data, off = pack(strs)
    for mode in (0, 5):
        e, eo = codec.encode_host(data, off, mode)
        o, oo2 = O.encode_batch(data, off, mode)
        assert np.array_equal(e, o) and np.array_equal(eo, oo2)
    h, ho = O.encode_batch(data, off, 0)
    d, do, st = codec.decode_host(h, ho)
    assert not st.any() and np.array_equal(d, data)
    # per-string mirrors of lsqpack_enc_enc_str / qenc_enc_str_size /
    # lsqpack_huff_decode
    for k in load("kat_enc_str.json")["enc_str"]:
        s = bytes.fromhex(k["str"])
        assert codec.enc_enc_str(3, s, dst_len=0x1000) == bytes.fromhex(k["out"])
    assert codec.enc_enc_str(3, b"aaa", dst_len=2) == -1
    r = codec.enc_enc_str(5, b"www.netbsd.org", first_byte=0xC0)
    assert r == O.enc_enc_str(5, b"www.netbsd.org", first_byte=0xC0)
    assert codec.enc_str_size(b"www.netbsd.org") == 11
    st, out, n_src = codec.huff_decode(bytes.fromhex("f1e3c2f51531a245cf64df"))
    assert st == 0 and out == b"www.netbsd.org" and n_src == 11
    st, out, _ = codec.huff_decode(b"\xff")
    assert st == 3
    st, out, _ = codec.huff_decode(bytes.fromhex("f1e3c2f51531a245cf64df"),
                                   dst_len=4)
    assert st == 2
    # ABI 1's 5-argument qhuff_huff_decode: a complete string, same results
    import ctypes as C
    import qhuff
    L = qhuff.lib()
    for src, dl in ((bytes.fromhex("f1e3c2f51531a245cf64df"), 64),
                    (b"\xff", 64),
                    (bytes.fromhex("f1e3c2f51531a245cf64df"), 4)):
        d = C.create_string_buffer(dl)
        rv = L.qhuff_huff_decode(codec._ctx, src, len(src), d, dl)
        st, out, n_src = codec.huff_decode(src, dst_len=dl)
        assert (rv.status, d.raw[:rv.n_dst], rv.n_src) == (st, out, n_src)


def test_host_path_pipelined_chunks(codec):
    """Batches large enough for the chunked host pipeline (8 MB chunks,
    several of them), with in_off[0] != 0 and invalid decode inputs."""
    import qhuff
    # ~44 MB of input: several 8 MB pipeline chunks, a ragged last one
    data, off = qhuff.synth_batch(1000003, seed=77, max_len=80)
    pad = 5
    data2 = np.concatenate([np.full(pad, 0x41, dtype=np.uint8), data])
    off2 = off + pad
    for mode in (0, 7):
        e, eo = codec.encode_host(data2, off2, mode)
        o, oo = O.encode_batch(data, off, mode)
        assert np.array_equal(eo, oo) and np.array_equal(e, o)
    h, ho = O.encode_batch(data, off, 0)
    h = h.copy()
    # corrupt every 97th string's last byte (most become invalid padding)
    for i in range(0, len(ho) - 1, 97):
        if ho[i + 1] > ho[i]:
            h[ho[i + 1] - 1] ^= 0x5A
    d, do, st = codec.decode_host(h, ho)
    od, odo, ost = O.decode_batch(h, ho)
    assert np.array_equal(st, ost) and np.array_equal(do, odo)
    assert np.array_equal(d, od)
    assert st.sum() > 100


def test_config4_full_size_sharded_round_trip(codec):
    """Config 4 at its full size: 16,777,216 strings (~604 MB) cut into 8
    byte-balanced shards (qhuff_shard_cuts, the per-GPU split of the 8-GPU
    run), each shard coded on cuda:0 through the in_off[0] != 0 path.
    Size-independent properties: the shard outputs stitched with their bases
    equal the unsharded encode byte for byte, and the unsharded output
    decodes back to the input with every status OK."""
    import qhuff
    n = 1 << 24
    data, off = qhuff.synth_batch(n, seed=0x5EED)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int32)).to(dev)
    del data
    full, full_off = codec.encode(d, o, 0)
    cuts = qhuff.shard_cuts(off, 8)
    assert cuts[0] == 0 and cuts[-1] == n
    fo = full_off.to(torch.int64)
    for k in range(8):
        s0, s1 = int(cuts[k]), int(cuts[k + 1])
        m = s1 - s0
        b = int(off[s1]) - int(off[s0])
        out = torch.empty(qhuff.encode_bound(b, m, 0), dtype=torch.uint8,
                          device=dev)
        oo = torch.empty(m + 1, dtype=torch.int32, device=dev)
        codec.encode_into(d, o[s0:], m, 0, out, oo)
        base = int(fo[s0])
        rel = fo[s0:s1 + 1] - base
        assert torch.equal(oo.to(torch.int64), rel)
        tot = int(rel[-1])
        assert torch.equal(out[:tot], full[base:base + tot])
        del out, oo
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    huff = full[:int(fo[-1])].contiguous()
    raw, roff, st = codec.decode(huff, full_off)
    torch.cuda.synchronize()
    assert codec.device_error() == 0
    assert not bool(st.any())
    assert torch.equal(roff, o)
    assert torch.equal(raw[:int(off[-1])], d)
