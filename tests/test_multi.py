"""One batch over several contexts (include/qhuff.h qhuff_*_batch_host_multi,
qhuff_*_batch_multi).

The path shards trivially (a string's output depends only on its own bytes
and the static table, lsqpack.c:5085-5195, 5234-5466): the C-ABI cuts a batch
by input bytes (qhuff_shard_cuts), runs each shard on its own context and
host thread, and stitches by the shards' bases.  Here G = 2 and 3 contexts
on one device (the box has one GPU; the code path is the same for G GPUs):
bit-exact against one single-context pass and against the oracle, on the
token batch, the reference's QIF corpora (big tiles, long strings) and
ragged edges (more contexts than strings, empty batches)."""
import os

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O
import qhuff

HERE = os.path.dirname(os.path.abspath(__file__))


def test_multi_rejects_bad_contexts():
    """(CPU) no context array, a null or a repeated context: QHUFF_EINVAL
    before any device call"""
    import ctypes as C
    L = qhuff.lib()
    off = np.zeros(2, dtype=np.uint32)
    buf = np.zeros(16, dtype=np.uint8)
    p = qhuff._np_ptr
    assert L.qhuff_encode_batch_host_multi(None, 1, p(buf), p(off), 1, 0,
                                           p(buf), p(off)) == qhuff.EINVAL
    nulls = (C.c_void_p * 2)(None, None)
    assert L.qhuff_decode_batch_host_multi(nulls, 2, p(buf), p(off), 1,
                                           p(buf), p(off), p(buf)) \
        == qhuff.EINVAL
    same = (C.c_void_p * 2)(1234, 1234)
    base = (C.c_uint64 * 3)()
    assert L.qhuff_encode_batch_multi(same, 2, None, 0, base, 1) \
        == qhuff.EINVAL
    assert L.qhuff_decode_batch_multi(same, 0, None, base, 1) == qhuff.EINVAL


@pytest.fixture(scope="module")
def codecs():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    cs = [qhuff.Codec(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


def _batches():
    from qhuff import workload
    tok = qhuff.synth_batch(300_000, seed=17)
    corpus = workload.corpus_batch(200_000, os.path.join(HERE, "golden",
                                                         "data"))
    return {"token": tok, "corpus": corpus}


@pytest.fixture(scope="module")
def batches():
    out = {}
    for k, (d, o) in _batches().items():
        h, ho = O.encode_batch(d, o, 0)
        out[k] = (d, o, h, ho)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("g", [2, 3])
@pytest.mark.parametrize("kind", ["token", "corpus"])
def test_host_multi_matches_single_pass(codecs, batches, g, kind):
    data, off, h, ho = batches[kind]
    one_e, one_eo = codecs[0].encode_host(data, off, 0)
    e, eo = qhuff.encode_host_multi(codecs[:g], data, off, 0)
    assert np.array_equal(eo, ho) and np.array_equal(e, h)
    assert np.array_equal(eo, one_eo) and np.array_equal(e, one_e)
    d, do, st = qhuff.decode_host_multi(codecs[:g], h, ho)
    assert not st.any()
    assert np.array_equal(do, off - off[0]) and np.array_equal(d, data)
    # a literal mode: framing bytes depend on each string alone too
    e7, eo7 = qhuff.encode_host_multi(codecs[:g], data, off, 7)
    s7, so7 = codecs[0].encode_host(data, off, 7)
    assert np.array_equal(eo7, so7) and np.array_equal(e7, s7)
    for c in codecs[:g]:
        assert c.device_error() == 0


@pytest.mark.gpu
def test_host_multi_rejects_and_edges(codecs):
    # invalid strings keep their status through the stitch
    import random
    rng = random.Random(3)
    strs = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 30)))
            for _ in range(5000)]
    off = np.zeros(len(strs) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strs], out=off[1:])
    data = np.frombuffer(b"".join(strs), dtype=np.uint8).copy()
    d, do, st = qhuff.decode_host_multi(codecs, data, off)
    want = [O.huff_decode(s) for s in strs]
    assert list(st) == [0 if w[0] == O.OK else 1 for w in want]
    for i, w in enumerate(want):
        assert bytes(d[do[i]:do[i + 1]]) == (w[1] if w[0] == O.OK else b"")
    # more contexts than strings, one string, none
    for n in (2, 1, 0):
        dd, oo = qhuff.synth_batch(n, seed=n) if n else (
            np.zeros(1, np.uint8), np.zeros(1, np.uint32))
        e, eo = qhuff.encode_host_multi(codecs, dd, oo, 0)
        h, ho = O.encode_batch(dd, oo, 0) if n else (np.zeros(0, np.uint8),
                                                      np.zeros(1, np.uint32))
        assert np.array_equal(eo, ho) and np.array_equal(e, h)


@pytest.mark.gpu
@pytest.mark.parametrize("g", [2, 3])
def test_device_multi_rebase(codecs, batches, g):
    """device-resident shards: each shard uploaded to its context's device,
    qhuff_*_batch_multi launches them all and rebases every shard's out_off
    on its device -- the concatenated outputs and the stitched offsets equal
    one single-context pass"""
    import torch
    data, off, h, ho = batches["corpus"]
    n = len(off) - 1
    cuts = qhuff.shard_cuts(off, g)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    shards, dsh = [], []
    for k in range(g):
        a, b = int(cuts[k]), int(cuts[k + 1])
        m = b - a
        so = off[a:b + 1].astype(np.int64)
        hs = ho[a:b + 1].astype(np.int64)
        shards.append(dict(
            in_=dev(data[so[0]:so[-1]]),
            in_off=dev((so - so[0]).astype(np.uint32).view(np.int32)),
            n=m, out=torch.empty(qhuff.encode_bound(int(so[-1] - so[0]), m, 0)
                                 + 16, dtype=torch.uint8, device="cuda"),
            out_off=torch.empty(m + 1, dtype=torch.int32, device="cuda"),
            stream=torch.cuda.Stream()))
        dsh.append(dict(
            in_=dev(h[hs[0]:hs[-1]]),
            in_off=dev((hs - hs[0]).astype(np.uint32).view(np.int32)),
            n=m, out=torch.empty(qhuff.decode_bound(int(hs[-1] - hs[0]), m)
                                 + 16, dtype=torch.uint8, device="cuda"),
            out_off=torch.empty(m + 1, dtype=torch.int32, device="cuda"),
            status=torch.empty(max(m, 1), dtype=torch.uint8, device="cuda"),
            stream=torch.cuda.Stream()))
    base = qhuff.batch_multi(codecs[:g], shards, True, 0)
    dbase = qhuff.batch_multi(codecs[:g], dsh, False)
    assert base[-1] == int(ho[-1]) and dbase[-1] == int(off[-1] - off[0])
    eo = np.concatenate([s["out_off"].cpu().numpy().view(np.uint32)[:-1]
                         for s in shards] + [[base[-1]]]).astype(np.uint32)
    assert np.array_equal(eo, ho)
    e = np.concatenate([s["out"][:base[k + 1] - base[k]].cpu().numpy()
                        for k, s in enumerate(shards)])
    assert np.array_equal(e, h)
    do = np.concatenate([s["out_off"].cpu().numpy().view(np.uint32)[:-1]
                         for s in dsh] + [[dbase[-1]]]).astype(np.uint32)
    assert np.array_equal(do, off - off[0])
    d = np.concatenate([s["out"][:dbase[k + 1] - dbase[k]].cpu().numpy()
                        for k, s in enumerate(dsh)])
    assert np.array_equal(d, data)
    assert not any(s["status"][:s["n"]].cpu().numpy().any() for s in dsh)
    for c in codecs[:g]:
        assert c.device_error() == 0
