"""The real-workload helpers behind bench.py's `workloads` leg
(qhuff/workload.py): the batches are what they claim
to be, and the tile-path shares follow the kernels' thresholds.  CPU only
(host arithmetic over offsets; the GPU parity of these batches is in
test_gpu_parity.py)."""
import os

import numpy as np

import _paths  # noqa: F401
import oracle_lib as O
import qhuff
from qhuff import workload as W

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def _shares(strs):
    data, off = W.pack(strs)
    h, ho = O.encode_batch(data, off, 0)
    return W.tile_shares(data, off, ho)


def test_corpus_batch_is_the_qif_strings_repeated():
    base = W.qif_strings([os.path.join(G, q) for q in W.QIF_NAMES])
    data, off = W.corpus_batch(len(base) + 10, G)
    assert len(off) == len(base) + 11
    got = [bytes(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
    assert got[:len(base)] == base and got[len(base):] == base[:10]


def test_alphabet_c_holds_long_codes():
    data, off = W.alphabet_c(1 << 12)
    assert len(off) == (1 << 12) + 1
    frac = np.isin(data, np.frombuffer(W.LONG_CODE_BYTES, np.uint8)).mean()
    assert 0.005 < frac < 0.05
    assert (W.RFC_LEN[data] > 13).any()


def test_rfc_lengths_match_the_oracle():
    assert [int(W.RFC_LEN[b]) for b in range(256)] == \
        [O.code_of(b)[1] for b in range(256)]


def test_token_batch_takes_the_fast_paths():
    data, off = qhuff.synth_batch(64 * 40, seed=9)
    h, ho = O.encode_batch(data, off, 0)
    sh = W.tile_shares(data, off, ho)
    assert sh["tiles"] == 40
    for k in ("decode_slow_tile_share", "decode_coop_tile_share",
              "encode_slow_tile_share", "encode_fallback_share",
              "encode_coop_tile_share", "decode_var_arena_share"):
        assert sh[k] == 0.0, k


def test_long_and_big_tiles_are_counted():
    short = [b"x" * 10] * 63
    # tile 0: a 300-byte string (cooperative decode, whole-wave payload
    # copy); tile 1: a 5,000-byte string (input past the stages); tile 2:
    # short strings only
    sh = _shares(short + [b"ab" * 150] + short + [b"q" * 5000] + short + [b"y"])
    assert sh["tiles"] == 3
    assert sh["decode_coop_tile_share"] == round(1 / 3, 4)
    assert sh["decode_slow_tile_share"] == round(1 / 3, 4)
    assert sh["encode_slow_tile_share"] == round(1 / 3, 4)
    assert sh["encode_coop_tile_share"] == round(1 / 3, 4)


def test_batch_needs_full():
    """qhuff_batch_needs_full (host only): the full kernel for a batch with a
    string above 128 bytes or a 64-string tile past the 3 KB stage (the
    kernels' own big-tile / long-string rules), not for the token batch."""
    import numpy as np
    import qhuff
    data, off = qhuff.synth_batch(1 << 14, seed=9)
    assert qhuff.batch_needs_full(off) == 0
    lens = np.diff(off.astype(np.int64))
    lens[700] = 129
    assert qhuff.batch_needs_full(np.concatenate([[0], np.cumsum(lens)])) == 1
    lens[700] = 128
    assert qhuff.batch_needs_full(np.concatenate([[0], np.cumsum(lens)])) == 0
    big = np.full(64, 48, dtype=np.int64)               # a 3,072-byte tile
    assert qhuff.batch_needs_full(np.concatenate([[0], np.cumsum(big)])) == 1
    assert qhuff.batch_needs_full(np.zeros(1, np.uint32)) == 0
