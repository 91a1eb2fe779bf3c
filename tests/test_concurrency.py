"""Forward progress and launch ordering.

* Two contexts on one GPU run full-size (1M-string) launches at the same time
  on two streams.  Each grid alone fills the GPU, so neither is co-resident
  while the other runs: tiles come from in-order tickets
  (qhuff_device.h Tickets), so both finish, bit-exact, with no device error.
* One context used from two streams (a device-pointer call on a caller
  stream, then the host path on the context's own stream, no sync between):
  the launches share one look-back workspace and are ordered by the
  context's last-launch event.
"""
import numpy as np
import pytest

import _paths  # noqa: F401
import oracle_lib as O


@pytest.fixture(scope="module")
def batch():
    import qhuff
    data, off = qhuff.synth_batch(1 << 20, seed=99)
    h, ho = O.encode_batch(data, off, 0)
    return data, off, h, ho


def _dev(a, torch):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.gpu
def test_two_contexts_concurrent_full_size(batch):
    import torch
    import qhuff
    data, off, h, ho = batch
    c1, c2 = qhuff.Codec(0), qhuff.Codec(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    d = _dev(data, torch)
    o = _dev(off.view(np.int32), torch)
    hd = _dev(h, torch)
    hod = _dev(ho.view(np.int32), torch)
    n = len(off) - 1
    outs = []
    torch.cuda.synchronize()
    for _ in range(3):
        res = []
        for c, s in ((c1, s1), (c2, s2)):
            eo = torch.empty(qhuff.encode_bound(len(data), n, 0),
                             dtype=torch.uint8, device="cuda")
            eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            do = torch.empty(qhuff.decode_bound(len(h), n), dtype=torch.uint8,
                             device="cuda")
            doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            st = torch.empty(n, dtype=torch.uint8, device="cuda")
            c.encode_into(d, o, n, 0, eo, eoo, s)
            c.decode_into(hd, hod, n, do, doo, st, s)
            res.append((eo, eoo, do, doo, st))
        outs.append(res)
    torch.cuda.synchronize()
    assert c1.device_error() == 0 and c2.device_error() == 0
    for res in outs:
        for eo, eoo, do, doo, st in res:
            eoo = eoo.cpu().numpy().view(np.uint32)
            assert np.array_equal(eoo, ho)
            assert np.array_equal(eo[:int(eoo[-1])].cpu().numpy(), h)
            assert np.array_equal(doo.cpu().numpy().view(np.uint32), off)
            assert not st.cpu().numpy().any()
            assert np.array_equal(do[:len(data)].cpu().numpy(), data)
    c1.close()
    c2.close()


@pytest.mark.gpu
def test_one_context_two_streams(batch):
    import torch
    import qhuff
    data, off, h, ho = batch
    c = qhuff.Codec(0)
    s = torch.cuda.Stream()
    d = _dev(data, torch)
    o = _dev(off.view(np.int32), torch)
    n = len(off) - 1
    torch.cuda.synchronize()
    for _ in range(2):
        eo = torch.empty(qhuff.encode_bound(len(data), n, 0), dtype=torch.uint8,
                         device="cuda")
        eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
        c.encode_into(d, o, n, 0, eo, eoo, s)          # caller stream
        ho2, hoo2 = c.encode_host(data, off, 0)          # own stream, no sync
        dr, droo, dst = c.decode_host(h, ho)             # own stream
        c.encode_into(d, o, n, 0, eo, eoo, s)          # caller stream again
        # per-string calls right behind it, no sync
        s1 = bytes(data[off[5]:off[6]])
        assert c.enc_enc_str(7, s1) == O.enc_enc_str(7, s1)
        e1 = O.huffman_enc(s1)
        st1, out1, n1 = c.huff_decode(e1)
        assert (st1, out1, n1) == (0, s1, len(e1))
        s.synchronize()
        assert np.array_equal(hoo2, ho) and np.array_equal(ho2, h)
        assert np.array_equal(droo, off) and not dst.any()
        assert np.array_equal(dr, data)
        eoo = eoo.cpu().numpy().view(np.uint32)
        assert np.array_equal(eoo, ho)
        assert np.array_equal(eo[:int(eoo[-1])].cpu().numpy(), h)
    assert c.device_error() == 0
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [100_000, 150_000, 196_700, 400_000])
def test_two_contexts_concurrent_small(n):
    """Two contexts on two streams, several rounds back to back, at batch
    sizes around one round of the grid (W = 3,072 waves on 256 CUs): spread
    launches (100k, 150k strings: at most one tile per wave) and ticket-group
    launches just past one and two rounds (196,700 strings = W + 1 tiles,
    400k), where every wave claims until a claim lands past the end -- so
    whichever workgroups are resident can fill a gap in any ticket group
    (VERDICT r03 item 6): no spin-limit error, bit-exact."""
    import torch
    import qhuff
    data, off = qhuff.synth_batch(n, seed=n)
    h, ho = O.encode_batch(data, off, 0)
    c1, c2 = qhuff.Codec(0), qhuff.Codec(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    d = _dev(data, torch)
    o = _dev(off.view(np.int32), torch)
    hd = _dev(h, torch)
    hod = _dev(ho.view(np.int32), torch)
    torch.cuda.synchronize()
    outs = []
    for _ in range(6):
        for c, s in ((c1, s1), (c2, s2)):
            eo = torch.empty(qhuff.encode_bound(len(data), n, 0),
                             dtype=torch.uint8, device="cuda")
            eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            do = torch.empty(qhuff.decode_bound(len(h), n), dtype=torch.uint8,
                             device="cuda")
            doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            st = torch.empty(n, dtype=torch.uint8, device="cuda")
            c.encode_into(d, o, n, 0, eo, eoo, s)
            c.decode_into(hd, hod, n, do, doo, st, s)
            outs.append((eo, eoo, do, doo, st))
    torch.cuda.synchronize()
    assert c1.device_error() == 0 and c2.device_error() == 0
    for eo, eoo, do, doo, st in outs:
        eoo = eoo.cpu().numpy().view(np.uint32)
        assert np.array_equal(eoo, ho)
        assert np.array_equal(eo[:int(eoo[-1])].cpu().numpy(), h)
        assert np.array_equal(doo.cpu().numpy().view(np.uint32), off)
        assert not st.cpu().numpy().any()
        assert np.array_equal(do[:len(data)].cpu().numpy(), data)
    c1.close()
    c2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("banks", ["1", "4"])
def test_two_contexts_share_slot_pool_big_tiles(banks):
    """both contexts WRITE the device's big-tile slot pool at
    once (qhuff_host.cpp with_slots): with one bank (QHUFF_SLOT_BANKS=1)
    they share it, ordered by its event; with four the second context takes
    the first's bank once (ordered), then the first gets a bank of its own.  The batch is the reference's
    QIF corpora (tiles whose 1,461-byte values overflow the 3 KB stages)
    with a 4 KB string every 5,000 strings, 400k strings (~2 grid rounds)
    -- full kernels pinned, so every launch codes big tiles through the
    pool; two contexts on two streams, several launches back to back.
    Their launches are ordered by the pool's event: bit-exact against the
    oracle, no device error."""
    import os
    import random
    import torch
    import qhuff
    from qhuff import workload
    here = os.path.dirname(os.path.abspath(__file__))
    data, off = workload.corpus_batch(400_000,
                                      os.path.join(here, "golden", "data"))
    strs = [bytes(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    rng = random.Random(5)
    for i in range(0, len(strs), 5000):
        strs[i] = bytes(rng.choice(b"abcdefghij-_/") for _ in range(4096))
    data, off = workload.pack(strs)
    n = len(off) - 1
    h, ho = O.encode_batch(data, off, 0)
    sh = workload.tile_shares(data, off, ho)
    assert sh["decode_slow_tile_share"] > 0 and sh["encode_slow_tile_share"] > 0
    env = {"QHUFF_KERNELS": "full", "QHUFF_SLOT_BANKS": banks}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c1, c2 = qhuff.Codec(0), qhuff.Codec(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    d = _dev(data, torch)
    o = _dev(off.view(np.int32), torch)
    hd = _dev(h, torch)
    hod = _dev(ho.view(np.int32), torch)
    torch.cuda.synchronize()
    outs = []
    for _ in range(3):
        for c, s in ((c1, s1), (c2, s2)):
            eo = torch.empty(qhuff.encode_bound(len(data), n, 0),
                             dtype=torch.uint8, device="cuda")
            eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            do = torch.empty(qhuff.decode_bound(len(h), n), dtype=torch.uint8,
                             device="cuda")
            doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            st = torch.empty(n, dtype=torch.uint8, device="cuda")
            c.encode_into(d, o, n, 0, eo, eoo, s)
            c.decode_into(hd, hod, n, do, doo, st, s)
            outs.append((eo, eoo, do, doo, st))
    torch.cuda.synchronize()
    assert c1.device_error() == 0 and c2.device_error() == 0
    assert c1.kernel_variant(qhuff.KIND_DECODE) == 1
    for eo, eoo, do, doo, st in outs:
        eoo = eoo.cpu().numpy().view(np.uint32)
        assert np.array_equal(eoo, ho)
        assert np.array_equal(eo[:int(eoo[-1])].cpu().numpy(), h)
        assert np.array_equal(doo.cpu().numpy().view(np.uint32), off)
        assert not st.cpu().numpy().any()
        assert np.array_equal(do[:len(data)].cpu().numpy(), data)
    c1.close()
    c2.close()


@pytest.mark.gpu
def test_more_contexts_than_pool_banks():
    """five contexts on five streams, full kernels, big tiles, launches in
    rotation: four get pool banks of their own, the fifth (past the cap of
    four) takes banks from the others, ordered by their events -- every
    output bit-exact, no device error"""
    import os
    import random
    import torch
    import qhuff
    from qhuff import workload
    here = os.path.dirname(os.path.abspath(__file__))
    data, off = workload.corpus_batch(200_000,
                                      os.path.join(here, "golden", "data"))
    strs = [bytes(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    rng = random.Random(9)
    for i in range(0, len(strs), 4000):
        strs[i] = bytes(rng.choice(b"klmnopq-_/") for _ in range(4096))
    data, off = workload.pack(strs)
    n = len(off) - 1
    h, ho = O.encode_batch(data, off, 0)
    old = os.environ.get("QHUFF_KERNELS")
    os.environ["QHUFF_KERNELS"] = "full"
    try:
        cs = [qhuff.Codec(0) for _ in range(5)]
    finally:
        if old is None:
            del os.environ["QHUFF_KERNELS"]
        else:
            os.environ["QHUFF_KERNELS"] = old
    ss = [torch.cuda.Stream() for _ in cs]
    d = _dev(data, torch)
    o = _dev(off.view(np.int32), torch)
    hd = _dev(h, torch)
    hod = _dev(ho.view(np.int32), torch)
    torch.cuda.synchronize()
    outs = []
    for _ in range(2):
        for c, s in zip(cs, ss):
            eo = torch.empty(qhuff.encode_bound(len(data), n, 0),
                             dtype=torch.uint8, device="cuda")
            eoo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            do = torch.empty(qhuff.decode_bound(len(h), n), dtype=torch.uint8,
                             device="cuda")
            doo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
            st = torch.empty(n, dtype=torch.uint8, device="cuda")
            c.encode_into(d, o, n, 0, eo, eoo, s)
            c.decode_into(hd, hod, n, do, doo, st, s)
            outs.append((eo, eoo, do, doo, st))
    torch.cuda.synchronize()
    for c in cs:
        assert c.device_error() == 0
    for eo, eoo, do, doo, st in outs:
        eoo = eoo.cpu().numpy().view(np.uint32)
        assert np.array_equal(eoo, ho)
        assert np.array_equal(eo[:int(eoo[-1])].cpu().numpy(), h)
        assert np.array_equal(doo.cpu().numpy().view(np.uint32), off)
        assert not st.cpu().numpy().any()
        assert np.array_equal(do[:len(data)].cpu().numpy(), data)
    for c in cs:
        c.close()
