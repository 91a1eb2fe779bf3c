"""Device memory per context: a context
allocates in proportion to what it runs.  Big-tile slots (48 KB per wave of
a launch's grid, qhuff_host.cpp with_slots) come from a per-context region
only for launches of at most 8 workgroups, allocated at the first such
launch, and from one pool per device for larger launches -- not, as in
round 4, 192 MB per context at qhuff_open.  Measured with hipMemGetInfo
(torch.cuda.mem_get_info) deltas, outputs checked against the oracle."""
import random

import numpy as np
import pytest
import torch

import _paths  # noqa: F401
import oracle_lib as O

MB = 1 << 20


def free_bytes():
    torch.cuda.synchronize()
    return torch.cuda.mem_get_info(0)[0]


@pytest.mark.gpu
def test_per_string_contexts_small():
    """16 contexts, each running the per-string entry points (and a small
    batch) as 16 per-thread shim contexts would: <= 16 MB of device memory
    each, round 4's eager slots alone were ~192 MB."""
    import qhuff
    warm = qhuff.Codec(0)                 # runtime, code objects, scratch
    warm.enc_enc_str(7, b"warm-up")
    warm.huff_decode(O.huffman_enc(b"warm-up"))
    rng = random.Random(4)
    strs = [bytes(rng.choice(b"abcdefgh-/.") for _ in range(rng.randrange(1, 60)))
            for _ in range(40)]
    # (and the host path, on two contexts: six streams, so the runtime's
    # hardware queues -- GPU_MAX_HW_QUEUES, device memory of their own that
    # later streams share -- exist before the measurement, whichever tests
    # ran before this one)
    warm2 = qhuff.Codec(0)
    for w in (warm, warm2):
        w.encode_host(*_pack(strs), 0)
    before = free_bytes()
    ctxs = [qhuff.Codec(0) for _ in range(16)]
    try:
        for c in ctxs:
            for s in strs[:8]:
                assert c.enc_enc_str(7, s) == O.enc_enc_str(7, s)
                h = O.huffman_enc(s)
                st, out, n_src = c.huff_decode(h)
                assert (st, out) == (qhuff.HUFF_DEC_OK, s)
            data, off = _pack(strs)
            g_out, g_off = c.encode_host(data, off, 0)
            o_out, o_off = O.encode_batch(data, off, 0)
            assert np.array_equal(g_off, o_off)
            assert np.array_equal(g_out, o_out[:o_off[-1]])
        used = before - free_bytes()
        assert used <= 16 * 16 * MB, used / MB
    finally:
        for c in ctxs:
            c.close()
        warm.close()
        warm2.close()


def _pack(strs):
    off = np.zeros(len(strs) + 1, np.uint32)
    off[1:] = np.cumsum([len(s) for s in strs])
    return np.frombuffer(b"".join(strs), np.uint8).copy(), off


@pytest.mark.gpu
def test_token_batch_contexts_share_slots():
    """Full-grid launches share the device's slot pool: after a first
    context has run a 1M-string token batch, a second context running the
    same batch allocates <= 16 MB of its own; both exact."""
    import qhuff
    data, off = qhuff.synth_batch(1 << 20, seed=2)
    h, ho = O.encode_batch(data, off, 0)
    n = len(off) - 1
    d_in = torch.from_numpy(data).cuda()
    d_off = torch.from_numpy(off.view(np.int32)).cuda()
    d_h = torch.from_numpy(h[:ho[-1]].copy()).cuda()
    d_ho = torch.from_numpy(ho.view(np.int32)).cuda()
    out = torch.empty(qhuff.encode_bound(len(data), n), dtype=torch.uint8,
                      device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    dout = torch.empty(qhuff.decode_bound(int(ho[-1]), n), dtype=torch.uint8,
                       device="cuda")
    doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")

    def run(c):
        c.encode_into(d_in, d_off, n, 0, out, oo)
        c.decode_into(d_h, d_ho, n, dout, doo, dst)
        torch.cuda.synchronize()
        assert np.array_equal(oo.cpu().numpy().view(np.uint32), ho)
        assert np.array_equal(out[:int(ho[-1])].cpu().numpy(), h[:ho[-1]])
        assert not dst.any().item()
        assert np.array_equal(dout[:len(data)].cpu().numpy(), data)

    first = qhuff.Codec(0)
    try:
        run(first)
        before = free_bytes()
        second = qhuff.Codec(0)
        try:
            run(second)
            used = before - free_bytes()
            assert used <= 16 * MB, used / MB
        finally:
            second.close()
    finally:
        first.close()


@pytest.mark.gpu
def test_alternating_contexts_get_own_banks():
    """Two contexts alternating full-grid launches (an encode stream and a
    decode stream): the second takes the first's pool bank once, then the
    first gets a bank of its own (one grid's slots, 48 KB a wave), so the
    two are not serialised on one bank; outputs exact throughout."""
    import qhuff
    data, off = qhuff.synth_batch(1 << 19, seed=3)
    h, ho = O.encode_batch(data, off, 0)
    n = len(off) - 1
    d_in = torch.from_numpy(data).cuda()
    d_off = torch.from_numpy(off.view(np.int32)).cuda()
    out = torch.empty(qhuff.encode_bound(len(data), n), dtype=torch.uint8,
                      device="cuda")
    oo = torch.empty(n + 1, dtype=torch.int32, device="cuda")

    def run(c):
        c.encode_into(d_in, d_off, n, 0, out, oo)
        torch.cuda.synchronize()
        assert np.array_equal(oo.cpu().numpy().view(np.uint32), ho)
        assert np.array_equal(out[:int(ho[-1])].cpu().numpy(), h[:ho[-1]])

    a, b = qhuff.Codec(0), qhuff.Codec(0)
    try:
        run(a)
        run(b)                            # takes a's bank: no new memory
        before = free_bytes()
        for _ in range(3):
            run(a)                        # a's bank was taken: a new one
            run(b)
        used = before - free_bytes()
        props = torch.cuda.get_device_properties(0)
        bank = props.multi_processor_count * 12 * 48 * 1024
        assert bank * 0.9 <= used <= bank + 16 * MB, (used / MB, bank / MB)
    finally:
        a.close()
        b.close()
