"""Registered caller buffers for the host-memory calls (include/qhuff.h
qhuff_host_register / qhuff_host_unregister).

A host call whose buffers lie in registered ranges moves them by DMA
directly instead of through the pinned stage: the same results, bit-exact,
whether the input side, the output side, both or neither is registered, on a
multi-chunk batch (several staging chunks, in-place offset rebase), the QIF
corpus with strings that fail to decode (statuses written in place), and a
batch sharded over several contexts (direct output deferred until the shard's
base is known)."""
import os

import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O
import qhuff

HERE = os.path.dirname(os.path.abspath(__file__))


def test_register_rejects_bad_arguments():
    """(CPU) null, zero bytes and unknown pointers: QHUFF_EINVAL, no device
    call"""
    L = qhuff.lib()
    a = np.zeros(64, dtype=np.uint8)
    assert L.qhuff_host_register(None, 64) == qhuff.EINVAL
    assert L.qhuff_host_register(qhuff._np_ptr(a), 0) == qhuff.EINVAL
    assert L.qhuff_host_unregister(qhuff._np_ptr(a)) == qhuff.EINVAL
    assert L.qhuff_host_unregister(None) == qhuff.EINVAL


@pytest.fixture(scope="module")
def codecs():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a GPU")
    cs = [qhuff.Codec(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


@pytest.fixture(scope="module")
def token():
    # ~30 MB: several 8 MB staging chunks
    d, o = qhuff.synth_batch(1_000_000, seed=29)
    h, ho = O.encode_batch(d, o, 0)
    return d, o, h, ho


@pytest.fixture(scope="module")
def corpus():
    from qhuff import workload
    d, o = workload.corpus_batch(300_000, os.path.join(HERE, "golden", "data"))
    h, ho = O.encode_batch(d, o, 0)
    # every 997th string garbled: decode statuses other than OK
    h = h.copy()
    rng = np.random.default_rng(5)
    for i in range(0, len(ho) - 1, 997):
        if ho[i + 1] > ho[i]:
            h[ho[i + 1] - 1] = rng.integers(0, 256)
    return d, o, h, ho


def _bufs(n, bound):
    return (np.zeros(bound, dtype=np.uint8), np.zeros(n + 1, dtype=np.uint32),
            np.zeros(max(n, 1), dtype=np.uint8))


@pytest.mark.gpu
def test_register_twice_and_unregister(codecs):
    a = np.zeros(1 << 20, dtype=np.uint8)
    assert qhuff.host_register(a) == qhuff.OK
    assert qhuff.host_register(a) == qhuff.EINVAL
    assert qhuff.host_unregister(a) == qhuff.OK
    assert qhuff.host_unregister(a) == qhuff.EINVAL


@pytest.mark.gpu
@pytest.mark.parametrize("side", ["both", "in", "out"])
def test_registered_token_roundtrip(codecs, token, side):
    d, o, h, ho = token
    n = len(o) - 1
    c = codecs[0]
    e, eo, _ = _bufs(n, qhuff.encode_bound(int(o[-1]), n, 0))
    q, qo, st = _bufs(n, qhuff.decode_bound(int(ho[-1]), n))
    ins = [d, o, h, ho] if side in ("both", "in") else []
    outs = [e, eo, q, qo, st] if side in ("both", "out") else []
    with qhuff.registered(*(ins + outs)):
        e2, eo2 = c.encode_host(d, o, 0, out=e, out_off=eo)
        assert np.array_equal(eo2, ho) and np.array_equal(e2, h)
        q2, qo2, st2 = c.decode_host(h, ho, out=q, out_off=qo, status=st)
        assert not st2.any()
        assert np.array_equal(qo2, o) and np.array_equal(q2, d)
    assert c.device_error() == 0


@pytest.mark.gpu
def test_registered_corpus_statuses(codecs, corpus):
    d, o, h, ho = corpus
    n = len(o) - 1
    c = codecs[0]
    ref_q, ref_qo, ref_st = c.decode_host(h, ho)
    assert ref_st.any()
    q, qo, st = _bufs(n, qhuff.decode_bound(int(ho[-1]), n))
    with qhuff.registered(h, ho, q, qo, st):
        q2, qo2, st2 = c.decode_host(h, ho, out=q, out_off=qo, status=st)
    assert np.array_equal(st2, ref_st)
    assert np.array_equal(qo2, ref_qo) and np.array_equal(q2, ref_q)
    e, eo, _ = _bufs(n, qhuff.encode_bound(int(o[-1]), n, 7))
    ref_e, ref_eo = O.encode_batch(d, o, 7)
    with qhuff.registered(d, o, e, eo):
        e2, eo2 = c.encode_host(d, o, 7, out=e, out_off=eo)
    assert np.array_equal(eo2, ref_eo) and np.array_equal(e2, ref_e)


@pytest.mark.gpu
@pytest.mark.parametrize("g", [2, 3])
def test_registered_multi(codecs, token, g):
    """sharded host calls: each shard's direct output waits for its base"""
    import ctypes as C
    d, o, h, ho = token
    n = len(o) - 1
    L = qhuff.lib()
    ctxs = (C.c_void_p * g)(*[x._ctx for x in codecs[:g]])
    p = qhuff._np_ptr
    e, eo, _ = _bufs(n, qhuff.encode_bound(int(o[-1]), n, 0))
    q, qo, st = _bufs(n, qhuff.decode_bound(int(ho[-1]), n))
    with qhuff.registered(d, o, h, ho, e, eo, q, qo, st):
        assert L.qhuff_encode_batch_host_multi(ctxs, g, p(d), p(o), n, 0,
                                               p(e), p(eo)) == qhuff.OK
        assert np.array_equal(eo, ho) and np.array_equal(e[:eo[-1]], h)
        assert L.qhuff_decode_batch_host_multi(ctxs, g, p(h), p(ho), n, p(q),
                                               p(qo), p(st)) == qhuff.OK
        assert not st[:n].any()
        assert np.array_equal(qo, o) and np.array_equal(q[:qo[-1]], d)


@pytest.mark.gpu
def test_registered_too_small_is_staged(codecs, token):
    """an output buffer registered with fewer bytes than the call's bound
    (here exactly the output) is not used for direct DMA: the call stages
    as before, same bytes"""
    d, o, h, ho = token
    n = len(o) - 1
    c = codecs[0]
    bound = qhuff.encode_bound(int(o[-1]), n, 0)
    e = np.zeros(bound, dtype=np.uint8)
    eo = np.zeros(n + 1, dtype=np.uint32)
    part = e[:int(ho[-1])]
    with qhuff.registered(d, o, part, eo):
        e2, eo2 = c.encode_host(d, o, 0, out=e, out_off=eo)
    assert np.array_equal(eo2, ho) and np.array_equal(e2, h)
