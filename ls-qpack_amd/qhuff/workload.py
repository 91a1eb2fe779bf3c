"""Real-workload batches and the kernels' tile-path shares (bench.py
--workloads).

* corpus_batch: the names and values of the reference's QIF corpora
  (tests/golden/data/*.qif, copies of /root/reference/test/qifs/*.qif:
  `name<TAB>value` lines, blank lines between header blocks, '#' comments)
  in wire order, repeated to n strings;
* alphabet_c: the synthetic batch with SURVEY 8(d)'s long-code alphabet C
  (token alphabet plus ~2 % of {1, 2, 6, 92, 141});
* tile_shares: which path each 64-string tile of a batch takes in the
  kernels, by the kernels' own rules (host arithmetic over the offsets; no
  device needed): slow tiles (input span or output past the 3 KB stages,
  qhuff_pipeline.h / qhuff_decode_impl.h), decode tiles whose arena slots are
  placed by input offset (a string above kFixMaxLen Huffman bytes), decode
  tiles with a string the whole wave decodes (above kCoopMin Huffman bytes,
  its bitmap in its own arena slot: qhuff_decode_impl.h coop_decode),
  encode tiles that fall back from the dense stream to
  per-string packing (the span's codes overflow the dense stream,
  qhuff_encode_impl.h dense_pass) and encode tiles with a payload the whole
  wave copies (above kEncCoopBits dense bits).
"""
import os

import numpy as np

from . import TOKEN_ALPHABET, synth_batch

# RFC 7541 Appendix B code lengths of bytes 0..255 (SURVEY.md Appendix A;
# the same data as csrc/qhuff_tables.h kLen)
RFC_LEN = np.array([
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,
    6, 10, 10, 12, 13, 6, 8, 11, 10, 10, 8, 11, 8, 6, 6, 6,
    5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8, 15, 6, 12, 10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8, 13, 19, 13, 14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5,
    6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7, 15, 11, 14, 13, 28,
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,
], dtype=np.int64)

QIF_NAMES = ("fb-req.qif", "fb-resp.qif", "long-codes.qif", "netbsd.qif")
LONG_CODE_BYTES = bytes([1, 2, 6, 92, 141])

# kernel constants the shares follow (qhuff_pipeline.h kStageCap,
# qhuff_decode_impl.h kFixMaxLen / kCoopMin,
# qhuff_encode_impl.h kDenseBits / kEncCoopBits)
STAGE = 3072
TILE = 64
FIX_MAX_LEN = (5 * (108 - 1)) // 8
COOP_MIN = 128
DENSE_BITS = 32 * (STAGE // 4 + 4 - 2)
ENC_COOP_BITS = 1024


def qif_strings(paths):
    """Every name and value of the QIF files, in file order."""
    out = []
    for p in paths:
        with open(p, "rb") as f:
            for line in f.read().split(b"\n"):
                if not line or line.startswith(b"#"):
                    continue
                name, _, value = line.partition(b"\t")
                out.append(name)
                out.append(value)
    return out


def pack(strings):
    off = np.zeros(len(strings) + 1, dtype=np.uint32)
    np.cumsum([len(s) for s in strings], out=off[1:])
    data = np.frombuffer(b"".join(strings), dtype=np.uint8).copy()
    return data, off


def corpus_batch(n, data_dir):
    """n strings: the QIF corpora's names and values in wire order,
    repeated (corpus order, not shuffled)."""
    base = qif_strings([os.path.join(data_dir, q) for q in QIF_NAMES])
    reps = -(-n // len(base))
    return pack((base * reps)[:n])


def alphabet_c(n, seed=0x9E3779B97F4A7C15):
    """SURVEY 8(d) alphabet C: token alphabet + ~2 % long-code bytes."""
    return synth_batch(n, seed=seed, alphabet=TOKEN_ALPHABET * 5
                       + LONG_CODE_BYTES)


def _tile_bounds(off):
    n = len(off) - 1
    t0 = np.arange(0, n, TILE, dtype=np.int64)
    t1 = np.minimum(t0 + TILE, n)
    return t0, t1


def _span(a, b):
    """16-byte aligned span of [a, b) (buffers 16-byte aligned)."""
    pa = a & ~15
    pb = (b + 15) & ~15
    return pa, pb


def tile_shares(data, off, hoff):
    """Fraction of tiles on each kernel path, for encode (input data/off,
    payload-mode output offsets hoff) and decode (input offsets hoff)."""
    off = off.astype(np.int64)
    hoff = hoff.astype(np.int64)
    t0, t1 = _tile_bounds(off)
    nt = len(t0)
    # ---- decode tiles ----
    a, b = hoff[t0], hoff[t1]
    pa, pb = _span(a, b)
    out_total = off[t1] - off[t0]
    dec_staged = (pb - pa) <= STAGE
    dec_fast = dec_staged & (out_total + 64 <= STAGE)
    hl = np.diff(hoff)
    max_hl = np.maximum.reduceat(hl, t0) if len(hl) else np.zeros(nt, np.int64)
    var_arena = dec_fast & (max_hl > FIX_MAX_LEN)
    # a cooperative string: above COOP_MIN Huffman bytes (its bitmap lives
    # in its own arena slot, qhuff_decode_impl.h coop_decode), in a staged
    # tile -- fast, or big and staged whole
    coop = dec_staged & (max_hl > COOP_MIN)
    # ---- encode tiles (payload mode) ----
    ea, eb = off[t0], off[t1]
    epa, epb = _span(ea, eb)
    enc_total = hoff[t1] - hoff[t0]
    enc_staged = (epb - epa) <= STAGE
    enc_fast = enc_staged & (enc_total + 64 <= STAGE)
    lens = RFC_LEN[data.astype(np.int64)] if len(data) else np.zeros(0, np.int64)
    plen = np.concatenate([[0], np.cumsum(lens)])
    dense_bits = plen[eb] - plen[epa]
    dense = enc_fast & (dense_bits + 64 <= DENSE_BITS)
    sbits = plen[off[1:]] - plen[off[:-1]]
    big = (np.maximum.reduceat(sbits, t0) if len(sbits)
           else np.zeros(nt, np.int64))
    enc_coop = dense & (big > ENC_COOP_BITS)
    f = lambda m: round(float(m.mean()), 4) if nt else 0.0
    hist = np.percentile(np.diff(off), [50, 90, 99, 100]) if len(off) > 1 \
        else [0, 0, 0, 0]
    return {
        "tiles": int(nt),
        "decode_slow_tile_share": f(~dec_fast),
        "decode_var_arena_share": f(var_arena),
        "decode_coop_tile_share": f(coop),
        "encode_slow_tile_share": f(~enc_fast),
        "encode_fallback_share": f(enc_fast & ~dense),
        "encode_coop_tile_share": f(enc_coop),
        "raw_len_p50_p90_p99_max": [int(x) for x in hist],
    }
