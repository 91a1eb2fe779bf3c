"""Multi-rank sharding: world-size-2 gloo runs on CPU.

Each rank takes its byte-balanced shard (qhuff_shard_cuts), codes it with
shard-local offsets, and rank outputs are stitched by adding shard bases.
The CPU variant codes shards with the oracle (this checks the host-side
partition / rebase logic); the gpu variant codes them with the HIP codec
on cuda:0 from both ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _paths  # noqa: F401
import oracle_lib as ol
import qhuff
from qhuff import shard


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n, seed=7):
    return qhuff.synth_batch(n, seed=seed, min_len=0, max_len=90)


def _code(kind, data, off, use_gpu):
    if not use_gpu:
        if kind == "enc":
            out, oo = ol.encode_batch(data, off, 7)
            return out, oo, None
        out, oo, st = ol.decode_batch(data, off)
        return out, oo, st
    c = qhuff.Codec(0)
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(np.ascontiguousarray(data) if len(data) else
                         np.zeros(1, np.uint8)).to(dev)
    o = torch.from_numpy(off.astype(np.uint32).view(np.int32)).to(dev)
    if kind == "enc":
        out, oo = c.encode(d, o, 7)
        st = None
    else:
        out, oo, st = c.decode(d, o)
        st = st.cpu().numpy()
    torch.cuda.synchronize()
    oo = oo.cpu().numpy().view(np.uint32)
    res = out[:int(oo[-1])].cpu().numpy(), oo, st
    assert c.device_error() == 0
    c.close()
    return res


def _worker(rank, world, port, n, use_gpu, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data, off = _batch(n)
        huff, hoff = ol.encode_batch(data, off, 0)
        res = {}
        for kind, d, o in (("enc", data, off), ("dec", huff, hoff)):
            cuts = shard.plan(o, world)
            sd, so, _ = shard.shard_view(d, o, cuts, rank)
            out, oo, st = _code(kind, sd, so, use_gpu)
            parts = [None] * world
            dist.all_gather_object(parts, (out, oo, st))
            res[kind] = (cuts, parts)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def _run(world, n, use_gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, use_gpu, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    data, off = _batch(n)
    huff, hoff = ol.encode_batch(data, off, 0)
    # encode: stitched shards == whole-batch oracle, bit for bit
    cuts, parts = res["enc"]
    out, oo = shard.merge([(p[0], p[1]) for p in parts])
    ref, ref_off = ol.encode_batch(data, off, 7)
    assert np.array_equal(oo, ref_off)
    assert np.array_equal(out, ref)
    # byte balance: every shard within one string of the ideal cut
    tot = int(off[-1])
    for r in range(1, world):
        b = int(off[cuts[r]])
        assert abs(b - r * tot / world) <= 90 + 1
    # decode
    cuts, parts = res["dec"]
    out, oo = shard.merge([(p[0], p[1]) for p in parts])
    st = np.concatenate([p[2] for p in parts])
    rref, rref_off, rst = ol.decode_batch(huff, hoff)
    assert np.array_equal(oo, rref_off)
    assert np.array_equal(out, rref)
    assert np.array_equal(st, rst)
    assert np.array_equal(out, data)


def test_shard_merge_local():
    data, off = _batch(1000)
    for world in (1, 2, 3, 8):
        cuts = shard.plan(off, world)
        parts = []
        for r in range(world):
            sd, so, s0 = shard.shard_view(data, off, cuts, r)
            assert s0 == cuts[r]
            parts.append(ol.encode_batch(sd, so, 5))
        out, oo = shard.merge(parts)
        ref, ref_off = ol.encode_batch(data, off, 5)
        assert np.array_equal(out, ref) and np.array_equal(oo, ref_off)


def test_shard_gloo_world2_cpu():
    _run(2, 3000, use_gpu=False)


@pytest.mark.gpu
def test_shard_gloo_world2_gpu():
    _run(2, 20000, use_gpu=True)
