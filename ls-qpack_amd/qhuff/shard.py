"""Host-side sharding of one string batch across G GPUs.

Strings are independent, so a batch splits into G contiguous, byte-balanced
shards (`qhuff_shard_cuts`); each rank codes its shard with shard-local
offsets and the outputs are stitched back by adding each shard's base (an
exclusive scan of G totals).  No collective touches the data path."""
import numpy as np

from . import shard_cuts


def shard_view(data, in_off, cuts, rank):
    """Rank `rank`'s shard: (bytes, local in_off uint32[k+1], first string).
    `data`/`in_off` are the whole batch (numpy); the returned bytes are a
    view, the offsets are rebased to start at 0."""
    s0, s1 = int(cuts[rank]), int(cuts[rank + 1])
    off = np.asarray(in_off, dtype=np.uint32)
    b0, b1 = int(off[s0]), int(off[s1])
    local = (off[s0:s1 + 1] - np.uint32(b0)).astype(np.uint32)
    return data[b0:b1], local, s0


def merge(parts):
    """parts: per-shard (out bytes, out_off uint32[k+1]) in rank order ->
    (out bytes, global out_off uint32[n+1])."""
    outs, offs = [], [np.zeros(1, dtype=np.uint64)]
    base = 0
    for out, off in parts:
        off = np.asarray(off, dtype=np.uint64)
        tot = int(off[-1]) - int(off[0])
        outs.append(np.asarray(out[int(off[0]):int(off[-1])], dtype=np.uint8))
        offs.append(off[1:] - off[0] + base)
        base += tot
    if base >= 1 << 32:
        raise OverflowError("merged output exceeds 32-bit offsets")
    return (np.concatenate(outs) if outs else np.zeros(0, np.uint8),
            np.concatenate(offs).astype(np.uint32))


def plan(in_off, world):
    """Cut points for `world` ranks (byte-balanced)."""
    return shard_cuts(np.asarray(in_off, dtype=np.uint32), world)
