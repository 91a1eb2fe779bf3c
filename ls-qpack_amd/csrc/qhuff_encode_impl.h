// qhuff_encode_impl.h -- the encode side of the kernels: dense pass, sizing,
// bit packing, slow tiles and the tile policy, shared by the batch kernel
// (qhuff_encode.hip) and the service kernel (qhuff_service.hip).  See
// qhuff_encode.hip for the algorithm.
#pragma once

#include "qhuff_pipeline.h"

// pending tiles: at 3 the tiles' outputs in registers spill (enc 91 vs 75
// us); the oldest parked in LDS instead still spilled 5 VGPRs in the dense
// pass (72.8 vs 65.5 us, profiles/r02_h); round 3, with the pending state
// slimmed and the next tile's loads issued after the dense pass, 2 VGPRs
// still spill: 68.3 vs 63.0 us (profiles/r03_i).  Then, with the wave
// pointer and the flushed tile wave-uniform (readfirstlane) and the
// flush's per-lane addresses rebuilt per flush instead of held, depth 3
// fits in 168 VGPRs with no spill: encode 0.964 of depth 2 (four pairs),
// look-back re-polls 0.83 -> 0.18 per tile (profiles/r03_e3)
#ifndef QH_ENC_DEPTH
#define QH_ENC_DEPTH 3
#endif

// QH_MT_REP 1: the dense pass's code table in 32 copies, copy c on LDS bank
// c, lane l reading copy l % 32 (dense_pass): the 64 lookups of a wave are
// bank-conflict-free (one copy: text bytes hit a few dozen entries of a
// 1 KB table, several to a bank), for 32 KB of LDS.  Off: with the round-4
// dense pass (codes of any length) it measured slower in same-box pairs.
#ifndef QH_MT_REP
#define QH_MT_REP 0
#endif

namespace qhuff {

constexpr int kEncInCap = kStageCap;          // staged input bytes per tile
constexpr int kEncOutCap = kStageCap;         // output stage bytes per tile
constexpr int kDenseWords = kStageCap / 4 + 4;  // dense code stream (words)
constexpr uint32_t kDenseBits = 32u * (kDenseWords - 2);
constexpr int kSpanChunks = kStageCap / 16;   // 16-byte chunks per staged span
static_assert(64 * kChunks <= kSpanChunks && 16 * kSpanChunks <= kEncOutCap,
              "dense pass: every row's lens / s0 store in bounds");

struct EncWave                                // one wave's private LDS region
{
    alignas(16) uint32_t in[kEncInCap / 4 + 4];
    alignas(16) uint32_t dense[kDenseWords];    // codes back to back, MSB first
    alignas(16) uint32_t out[kEncOutCap / 4];   // byte code lengths until emit
    uint32_t s0[kSpanChunks];                   // dense offset of each chunk
};

struct EncSmem
{
    static constexpr bool kMtRep = QH_MT_REP;
    u32x2 enc[257];
    uint32_t mt[256];                // dense pass: mt_entry(code, len)
    uint32_t mtr[kMtRep ? 256 * 32 : 1];   // mt, 32 copies: [byte][copy]
    uint8_t len[256];
    EncWave w[kWaves];
    BlockTickets tk;                 // the workgroup's first tickets
};

// source of aligned input dwords: LDS stage or global
struct EncLds
{
    const QH_LDS uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};
struct EncGlb
{
    const QH_GLB uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};

// MSB-first bit packer writing straight to global memory (slow path).
// Words are flushed as big-endian dwords at 4-byte aligned positions;
// `lo`..`hi` are the bytes this string owns.
struct PackGlb
{
    uint8_t *out;                            // 4-byte aligned
    __device__ __forceinline__ void word(uint32_t wpos, uint32_t be,
                                         uint32_t lo, uint32_t hi) const
    {
        if (wpos >= lo && wpos + 4 <= hi)
            *(QH_GLB uint32_t *) (out + wpos) = bswap32(be);
        else
            for (int k = 0; k < 4; ++k)
            {
                uint32_t p = wpos + k;
                if (p >= lo && p < hi)
                    out[p] = (uint8_t) (be >> (24 - 8 * k));
            }
    }
};

template <class Sink>
struct Packer
{
    Sink sink;
    uint64_t acc;          // pending bits, left-aligned
    uint32_t nbits;        // bits in acc, counting the lead-in bytes
    uint32_t wpos, lo, hi;

    __device__ __forceinline__ void init(uint32_t start, uint32_t end)
    {
        lo = start;
        hi = end;
        wpos = start & ~3u;
        nbits = 8u * (start & 3);
        acc = 0;
    }
    __device__ __forceinline__ void put(uint32_t code, uint32_t len)
    {
        // len == 0 is a no-op (masked byte)
        const uint64_t v = len ? (uint64_t) code << (64 - nbits - len) : 0;
        acc |= v;
        nbits += len;
        if (nbits >= 32)
        {
            sink.word(wpos, (uint32_t) (acc >> 32), lo, hi);
            acc <<= 32;
            nbits -= 32;
            wpos += 4;
        }
    }
    // EOS-prefix padding to a byte boundary, then flush (lsqpack.c:5171-5189)
    __device__ __forceinline__ void finish()
    {
        uint32_t pad = (8 - (nbits & 7)) & 7;
        acc |= (uint64_t) ((1u << pad) - 1) << (64 - nbits - pad);
        nbits += pad;
        while (nbits > 0)
        {
            sink.word(wpos, (uint32_t) (acc >> 32), lo, hi);
            acc <<= 32;
            nbits = nbits > 32 ? nbits - 32 : 0;
            wpos += 4;
        }
    }
};

// HPACK prefixed-integer byte count (lsqpack_val2len, lsqpack.c:767-783)
__device__ __forceinline__ uint32_t
int_len(uint32_t v, uint32_t prefix)
{
    uint32_t mask = (1u << prefix) - 1;
    if (v < mask)
        return 1;
    v -= mask;
    uint32_t n = 2;
    while (v >= 128)
    {
        v >>= 7;
        ++n;
    }
    return n;
}

// valid-byte mask (4 bits) of dword d for a string [rs, re), re > rs
__device__ __forceinline__ uint32_t
byte_mask(uint32_t d, uint32_t d0, uint32_t dl, uint32_t rs, uint32_t re)
{
    uint32_t m = 0xfu;
    m &= (d == d0) ? (0xfu << (rs & 3)) : 0xfu;
    m &= (d == dl) ? (0xfu >> (3 - ((re - 1) & 3))) : 0xfu;
    return m;
}

// 4-bit valid-byte mask -> byte mask (0xff per set bit)
__device__ __forceinline__ uint32_t
mask_bytes(uint32_t m)
{
    return (m & 1 ? 0xffu : 0u) | (m & 2 ? 0xff00u : 0u)
         | (m & 4 ? 0xff0000u : 0u) | (m & 8 ? 0xff000000u : 0u);
}

__device__ __forceinline__ uint32_t
len4(uint32_t w, const QH_LDS uint8_t *s_len)
{
    return s_len[w & 0xff] | (s_len[(w >> 8) & 0xff] << 8)
         | (s_len[(w >> 16) & 0xff] << 16) | (s_len[w >> 24] << 24);
}

// sum of code lengths over bytes [rs, re) (positions relative to the source):
// two dwords per iteration, four lengths packed per dword, masked and summed
// with v_sad_u8
template <class Src>
__device__ __forceinline__ uint32_t
code_bits(const Src &src, uint32_t rs, uint32_t re, const QH_LDS uint8_t *s_len)
{
    uint32_t bits = 0;
    if (re == rs)
        return 0;
    const uint32_t d0 = rs >> 2, dl = (re - 1) >> 2;
    for (uint32_t d = d0; d <= dl; d += 2)
    {
        const bool two = d + 1 <= dl;
        const uint32_t w0 = src.dw(d);
        const uint32_t w1 = two ? src.dw(d + 1) : 0u;
        const uint32_t p0 = len4(w0, s_len), p1 = len4(w1, s_len);
        const uint32_t m0 = mask_bytes(byte_mask(d, d0, dl, rs, re));
        const uint32_t m1 = two ? mask_bytes(byte_mask(d + 1, d0, dl, rs, re)) : 0u;
        bits = __builtin_amdgcn_sad_u8(p0 & m0, 0u, bits);
        bits = __builtin_amdgcn_sad_u8(p1 & m1, 0u, bits);
    }
    return bits;
}

template <class Src, class Sink>
__device__ __forceinline__ void
pack_string(const Src &src, uint32_t rs, uint32_t re, bool raw,
            const QH_LDS u32x2 *s_enc, Packer<Sink> &pk)
{
    if (re == rs)
        return;
    const uint32_t d0 = rs >> 2, dl = (re - 1) >> 2;
    for (uint32_t d = d0; d <= dl; ++d)
    {
        const uint32_t w = src.dw(d);
        const uint32_t m = byte_mask(d, d0, dl, rs, re);
        u32x2 e[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
        {
            const uint32_t c = (w >> (8 * b)) & 0xff;
            const u32x2 t = s_enc[c];
            e[b].x = raw ? c : t.x;
            e[b].y = raw ? 8u : t.y;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b)
            pk.put(e[b].x, (m >> b) & 1 ? e[b].y : 0u);
    }
}

// ---- bit packing into an LDS output stage --------------------------------
//
// The stage holds the tile's output in byte order (byte-swapped big-endian
// words), zeroed before packing; bits are OR-ed in at their positions, so
// neighbouring strings (which share boundary words) need no coordination.

// OR the `len` (<= 32) low bits of v into the stream at bit `pos`
__device__ __forceinline__ void
or_bits(QH_LDS uint32_t *st, uint32_t pos, uint32_t v, uint32_t len)
{
    const uint32_t w = pos >> 5, o = pos & 31;
    uint64_t x = len ? ((uint64_t) v << (64 - len)) : 0ull;   // left-aligned
    x >>= o;
    __hip_atomic_fetch_or(&st[w], bswap32((uint32_t) (x >> 32)),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&st[w + 1], bswap32((uint32_t) x),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// codes of the (masked) bytes of one input dword
__device__ __forceinline__ void
codes4(uint32_t w, uint32_t m, bool raw, const QH_LDS u32x2 *s_enc,
       uint32_t (&c)[4], uint32_t (&l)[4])
{
#pragma unroll
    for (int b = 0; b < 4; ++b)
    {
        const uint32_t ch = (w >> (8 * b)) & 0xff;
        const u32x2 t = s_enc[ch];
        const bool on = (m >> b) & 1;
        c[b] = on ? (raw ? ch : t.x) : 0u;
        l[b] = on ? (raw ? 8u : t.y) : 0u;
    }
}

// concatenation of four codes of at most 32 bits in total
__device__ __forceinline__ uint32_t
cat4(const uint32_t (&c)[4], const uint32_t (&l)[4])
{
    uint32_t v = c[0];
    v = (l[1] ? v << l[1] : v) | c[1];
    v = (l[2] ? v << l[2] : v) | c[2];
    v = (l[3] ? v << l[3] : v) | c[3];
    return v;
}

// E2 / E3 payload of bytes [rs, re) of the LDS input (string per lane), from
// bit `pos`; four input bytes per step, their codes concatenated and OR-ed
// in at once when they fit 32 bits (a wave-uniform branch takes the others
// code by code).  Returns the end position.
__device__ __forceinline__ uint32_t
pack_bits(const QH_LDS uint32_t *in, uint32_t rs, uint32_t re, bool raw,
          const QH_LDS u32x2 *s_enc, QH_LDS uint32_t *st, uint32_t pos)
{
    if (re == rs)
        return pos;
    const uint32_t d0 = rs >> 2, dl = (re - 1) >> 2;
    for (uint32_t d = d0; d <= dl; d += 2)
    {
        const bool two = d + 1 <= dl;
        const uint32_t w0 = in[d];
        const uint32_t w1 = two ? in[d + 1] : 0u;
        uint32_t c0[4], l0[4], c1[4], l1[4];
        codes4(w0, byte_mask(d, d0, dl, rs, re), raw, s_enc, c0, l0);
        codes4(w1, two ? byte_mask(d + 1, d0, dl, rs, re) : 0u, raw, s_enc,
               c1, l1);
        const uint32_t L0 = l0[0] + l0[1] + l0[2] + l0[3];
        const uint32_t L1 = l1[0] + l1[1] + l1[2] + l1[3];
        if (__builtin_amdgcn_ballot_w64(L0 > 32 || L1 > 32))
        {
#pragma unroll
            for (int b = 0; b < 4; ++b)
            {
                or_bits(st, pos, c0[b], l0[b]);
                pos += l0[b];
            }
#pragma unroll
            for (int b = 0; b < 4; ++b)
            {
                or_bits(st, pos, c1[b], l1[b]);
                pos += l1[b];
            }
        }
        else
        {
            or_bits(st, pos, cat4(c0, l0), L0);
            pos += L0;
            or_bits(st, pos, cat4(c1, l1), L1);
            pos += L1;
        }
    }
    return pos;
}

// literal framing (lsqpack.c:852-854, 862-864, 819-836): H bit + the length
// as an HPACK integer with a `mode`-bit prefix, at bit `pos`; returns the
// position after it
__device__ __forceinline__ uint32_t
emit_prefix(QH_LDS uint32_t *st, uint32_t pos, uint32_t mode, bool huff,
            uint32_t plen)
{
    const uint32_t mask = (1u << mode) - 1, first = huff ? (1u << mode) : 0;
    if (plen < mask)
    {
        or_bits(st, pos, first | plen, 8);
        return pos + 8;
    }
    or_bits(st, pos, first | mask, 8);
    pos += 8;
    uint32_t v = plen - mask;
    while (v >= 128)
    {
        or_bits(st, pos, 0x80 | (v & 0x7f), 8);
        pos += 8;
        v >>= 7;
    }
    or_bits(st, pos, v, 8);
    return pos + 8;
}

// literal framing + payload + EOS-prefix padding into the LDS stage, from
// byte `start`, string per lane (lsqpack.c:839-876, 5171-5189)
__device__ __forceinline__ void
emit_bits(const QH_LDS uint32_t *in, uint32_t rs, uint32_t re, uint32_t mode,
          bool huff, uint32_t plen, const QH_LDS u32x2 *s_enc,
          QH_LDS uint32_t *st, uint32_t start)
{
    uint32_t pos = 8 * start;
    if (mode)
        pos = emit_prefix(st, pos, mode, huff, plen);
    pos = pack_bits(in, rs, re, !huff, s_enc, st, pos);
    const uint32_t pad = (8 - (pos & 7)) & 7;
    if (pad)
        or_bits(st, pos, (1u << pad) - 1, pad);
}

// literal framing (lsqpack.c:852-854, 862-864, 819-836): H bit + prefixed
// length, then the payload (slow path, straight to global memory)
template <class Src, class Sink>
__device__ __forceinline__ void
emit_string(const Src &src, uint32_t rs, uint32_t re, uint32_t mode,
            bool huff, uint32_t plen, const QH_LDS u32x2 *s_enc,
            Packer<Sink> &pk)
{
    if (mode)
    {
        uint32_t mask = (1u << mode) - 1, first = huff ? (1u << mode) : 0;
        if (plen < mask)
            pk.put(first | plen, 8);
        else
        {
            pk.put(first | mask, 8);
            uint32_t v = plen - mask;
            while (v >= 128)
            {
                pk.put(0x80 | (v & 0x7f), 8);
                v >>= 7;
            }
            pk.put(v, 8);
        }
    }
    pack_string(src, rs, re, !huff, s_enc, pk);
    pk.finish();
}

// per-string sizing result
struct EncSize
{
    uint32_t size, plen;
    bool huff;
};

// E1 bits -> output size and the E3 choice (strict <, lsqpack.c:848)
__device__ __forceinline__ EncSize
size_from_bits(uint32_t mode, uint32_t bits, uint32_t len)
{
    EncSize z;
    const uint32_t hb = (bits + 7) >> 3;
    z.huff = true;
    z.plen = 0;
    if (mode == 0)
        z.size = hb;
    else
    {
        z.huff = hb < len;
        z.plen = z.huff ? hb : len;
        z.size = int_len(z.plen, mode) + z.plen;
    }
    return z;
}

template <class Src>
__device__ __forceinline__ EncSize
size_string(uint32_t mode, const Src &src, uint32_t rs, uint32_t re,
            const QH_LDS uint8_t *s_len)
{
    return size_from_bits(mode, code_bits(src, rs, re, s_len), re - rs);
}

// ---- byte-parallel dense pass ------------------------------------------------

// OR the right-aligned len-bit value v (len <= 32; v = 0 when len = 0) into
// the dense stream at bit pos (words hold their bits MSB first, unswapped)
__device__ __forceinline__ void
dense_or(QH_LDS uint32_t *dense, uint32_t pos, uint32_t v, uint32_t len)
{
    const uint32_t l = v << ((32u - len) & 31);
    const uint64_t x = ((uint64_t) l << 32) >> (pos & 31);
    // past the stream: both ORs land on its last two words (the tile then
    // falls back; no lane branches -- each one cost exec-mask traffic)
    const uint32_t w = min(pos >> 5, (uint32_t) kDenseWords - 2);
    const uint32_t hi = (uint32_t) (x >> 32), lo = (uint32_t) x;
    __hip_atomic_fetch_or(&dense[w], hi, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dense[w + 1], lo, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}

// QH_MT_LOW 1: the dense pass's table entry is code[26:0] << 5 | len (len
// in the low bits: a group's four lengths gathered by two byte permutes,
// and a shift takes the entry itself as its amount); 0: len << 27 | code.
// Encode lab: dense pass 4.49k -> 3.99k cycles per tile at 12 waves/CU;
// kernel 0.973 in 3 same-box pairs, corpus encode 0.978 (profiles/r05_low)
#ifndef QH_MT_LOW
#define QH_MT_LOW 1
#endif
__device__ __forceinline__ uint32_t
mt_entry(uint32_t code, uint32_t len)
{
    return QH_MT_LOW ? ((code & 0x7ffffffu) << 5) | len
                     : (code & 0x7ffffffu) | (len << 27);
}
__device__ __forceinline__ uint32_t
mt_code(uint32_t m)
{
    return QH_MT_LOW ? m >> 5 : m & 0x7ffffffu;
}
__device__ __forceinline__ uint32_t
mt_len(uint32_t m)
{
    return QH_MT_LOW ? m & 31u : m >> 27;
}
// the four lengths of entries a..d as bytes
__device__ __forceinline__ uint32_t
mt_lens4(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
#if QH_MT_LOW
    const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm(d, c, 0x04000c0cu);
    return (lo | hi) & 0x1f1f1f1fu;
#else
    return (a >> 27) | ((b >> 27) << 8) | ((c >> 27) << 16) | ((d >> 27) << 24);
#endif
}

// dense pass: a lane's 4-byte groups in pairs, one 64-bit value and three
// ORs per pair instead of two per group (encode lab: dense pass 5.27k ->
// 4.46k cycles per tile at 12 waves/CU; kernel 0.990 of the per-group ORs
// in 3 same-box pairs, corpus encode 0.976, profiles/r05_dp; skipping the
// third OR where it is zero: 4.67k, 0.994)
#ifndef QH_DENSE_PAIR
#define QH_DENSE_PAIR 1
#endif

// OR the right-aligned len-bit value v (len <= 64) into the dense stream at
// bit pos: three words (past the stream: its last three)
__device__ __forceinline__ void
dense_or64(QH_LDS uint32_t *dense, uint32_t pos, uint64_t v, uint32_t len)
{
    const uint64_t x = v << ((64u - len) & 63);
    const uint32_t sh = pos & 31;
    const uint32_t w = min(pos >> 5, (uint32_t) kDenseWords - 3);
    const uint32_t w0 = (uint32_t) (x >> (32 + sh));
    const uint32_t w1 = (uint32_t) (x >> sh);
    const uint32_t w2 = sh ? (uint32_t) (x << (32 - sh)) : 0u;
#ifdef QH_TIME_DENSE_STORE                   // timing builds only: wrong output
    if (QH_TIME_DENSE_STORE == 1)
    {
        dense[w] = w0;
        dense[w + 1] = w1;
        dense[w + 2] = w2;
    }
    return;
#endif
    __hip_atomic_fetch_or(&dense[w], w0, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dense[w + 1], w1, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_or(&dense[w + 2], w2, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Byte-parallel pass over the tile's staged chunks (lane l holds span chunks
// l, l + 64, l + 128): code lengths per byte (u8, into the out stage), the
// dense offset of every chunk (s0) and the codes of all span bytes back to
// back in `dense` -- the bytes around the tile's strings included (their
// codes shift every offset by the same amount).  Codes of any length (a
// stream longer than `dense` is caught by the codec's size check: its ORs
// pile up on the last two words).
template <bool Rep>
__device__ __forceinline__ void
dense_pass(uint32_t n16, const QH_LDS uint32_t *mt, QH_LDS EncWave *wv)
{
    const uint32_t lane = lane_id();
    QH_LDS u32x4 *d4 = (QH_LDS u32x4 *) wv->dense;
    for (uint32_t i = lane; i < (uint32_t) kDenseWords / 4; i += 64)
        d4[i] = (u32x4){0, 0, 0, 0};
    wave_sync();
    QH_LDS u32x4 *lens4 = (QH_LDS u32x4 *) wv->out;
    uint32_t carry = 0;
    // (the three rows' stage chunks read up front, one LDS round trip: enc
    // 66.1 vs 65.4 us, profiles/r02_l/ab_rows_first.txt)
#pragma unroll
    for (int k = 0; k < kChunks; ++k)
    {
        // every row is coded (no exit for short spans): straight-line code
        // lets the rows' lookups overlap; chunks past the span read its last
        // staged chunk again, coded past its end and never read
        const uint32_t c = lane + 64u * k;
        const uint32_t last = n16 ? n16 - 1 : 0;
        const u32x4 w = ((const QH_LDS u32x4 *) wv->in)[c < last ? c : last];
        const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
        uint32_t m[16];
        // (Rep) this lane's copy, rebuilt per row by an opaque instruction:
        // left to itself the compiler keeps it live through the tile loop,
        // and at 168 VGPRs that spills the sizing phase's offsets
        uint32_t copy = 0;
        if (Rep)
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\t"
                         "v_mbcnt_hi_u32_b32 %0, -1, %0\n\t"
                         "v_and_b32 %0, 31, %0" : "=v"(copy));
#pragma unroll
        for (int j = 0; j < 16; ++j)
        {
            const uint32_t b = (wd[j >> 2] >> (8 * (j & 3))) & 0xffu;
            m[j] = mt[Rep ? (b << 5) | copy : b];
        }
        uint32_t lp[4], G[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
        {
            lp[g] = mt_lens4(m[4 * g], m[4 * g + 1], m[4 * g + 2], m[4 * g + 3]);
            G[g] = __builtin_amdgcn_sad_u8(lp[g], 0u, 0u);
        }
        const uint32_t T = G[0] + G[1] + G[2] + G[3];
        const uint32_t incl = wave_incl_scan(T);
        const uint32_t p0 = carry + incl - T;
        carry += read_lane(incl, 63);
        // c < kSpanChunks always: rows past the span store too (never read)
        lens4[c] = (u32x4){lp[0], lp[1], lp[2], lp[3]};
        wv->s0[c] = p0;
        uint32_t pos = p0;
#if QH_DENSE_PAIR
        // groups in pairs: one 64-bit value, three ORs instead of four
        if (!__builtin_amdgcn_ballot_w64((G[0] > 32) | (G[1] > 32) | (G[2] > 32)
                                         | (G[3] > 32)))
        {
#pragma unroll
            for (int h = 0; h < 2; ++h)
            {
                uint32_t v[2];
#pragma unroll
                for (int e = 0; e < 2; ++e)
                {
                    const int g = 2 * h + e;
                    uint32_t x = mt_code(m[4 * g]);
#pragma unroll
                    for (int j = 1; j < 4; ++j)
                        x = (x << (QH_MT_LOW ? m[4 * g + j] & 31u : mt_len(m[4 * g + j])))
                          | mt_code(m[4 * g + j]);
                    v[e] = x;
                }
                const uint32_t n = G[2 * h] + G[2 * h + 1];
                dense_or64(wv->dense, pos, ((uint64_t) v[0] << G[2 * h + 1]) | v[1],
                           n);
                pos += n;
            }
            continue;
        }
#endif
#pragma unroll
        for (int g = 0; g < 4; ++g)
        {
            uint32_t cd[4], L[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
            {
                cd[j] = mt_code(m[4 * g + j]);
                L[j] = mt_len(m[4 * g + j]);
            }
            if (__builtin_amdgcn_ballot_w64(G[g] > 32))
            {
                // (rare) a code of 28 or 30 bits: its ones above bit 26
                if (__builtin_amdgcn_ballot_w64(((lp[g] + 0x64646464u)
                                                 & 0x80808080u) != 0))
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        cd[j] |= L[j] > 27 ? (0xffffffffu >> (32 - L[j]))
                                                 & ~0x7ffffffu
                                           : 0u;
                const uint32_t a = L[0] + L[1], b = L[2] + L[3];
                if (__builtin_amdgcn_ballot_w64((a > 32) | (b > 32)))
                {
                    // (rare) codes above 16 bits: one OR per code
                    dense_or(wv->dense, pos, cd[0], L[0]);
                    dense_or(wv->dense, pos + L[0], cd[1], L[1]);
                    dense_or(wv->dense, pos + a, cd[2], L[2]);
                    dense_or(wv->dense, pos + a + L[2], cd[3], L[3]);
                }
                else
                {
                    // a lane's four codes exceed 32 bits: two pairs
                    dense_or(wv->dense, pos, (cd[0] << L[1]) | cd[1], a);
                    dense_or(wv->dense, pos + a, (cd[2] << L[3]) | cd[3], b);
                }
            }
            else
            {
                uint32_t v = (cd[0] << L[1]) | cd[1];
                v = (v << L[2]) | cd[2];
                v = (v << L[3]) | cd[3];
                dense_or(wv->dense, pos, v, G[g]);
            }
            pos += G[g];
        }
    }
}

// dense offset of span byte p (p <= 16 * n16): the offset of the chunk
// holding byte p - 1 plus the code lengths of that chunk's bytes before p
__device__ __forceinline__ uint32_t
dense_at(const QH_LDS EncWave *wv, uint32_t p)
{
    const uint32_t k = (p ? p - 1 : 0) >> 4;
    const uint32_t nb = p - 16 * k;                      // 0..16 bytes
    const u32x4 l = ((const QH_LDS u32x4 *) wv->out)[k];
    const uint32_t ld[4] = {l.x, l.y, l.z, l.w};
    uint32_t s = wv->s0[k];
#pragma unroll
    for (int j = 0; j < 4; ++j)
    {
        const uint32_t cj = nb > 4u * j ? min(nb - 4u * j, 4u) : 0u;
        const uint32_t mk = cj >= 4 ? 0xffffffffu : ((1u << (8 * cj)) - 1);
        s = __builtin_amdgcn_sad_u8(ld[j] & mk, 0u, s);
    }
    return s;
}

// the nb (> 0) dense bits from bit s to the byte-aligned bit d of the output
// stage (byte order): one 32-bit window of the dense stream per output word;
// plain stores for the words the string owns whole, OR for its first and
// last word (shared with framing, padding and the neighbours)
template <bool Mid = true>
__device__ __forceinline__ void
copy_dense(const QH_LDS uint32_t *dense, uint32_t s, uint32_t nb,
           QH_LDS uint32_t *st, uint32_t d)
{
    const uint32_t e = d + nb;
    const uint32_t w0 = d >> 5, wl = (e - 1) >> 5, od = d & 31;
    const uint32_t tailm = 0xffffffffu << (31 - ((e - 1) & 31));
    // Every read of the first word, the first trip and the last word is
    // issued before any write (a wave's LDS operations run in order, so a
    // read behind a write waits for it): a string of up to 6 output words
    // costs one LDS round trip.  The words the string owns whole (w0 + 1 ..
    // wl - 1) by plain stores, four per trip with the trip's reads issued
    // together; its first and last words, shared with its neighbours and its
    // framing / padding, by OR.
    // output word w0 + k (k >= 1) <- the window at dense bit s - od + 32 k
    const uint32_t q0 = s >> 5, os = s & 31;
    const uint32_t x1 = s - od + 32, sh = x1 & 31, q = x1 >> 5;
    const uint32_t nmid = wl > w0 ? wl - w0 - 1 : 0u;
    auto win = [&](uint32_t a, uint32_t b) -> uint32_t {
        return sh ? __builtin_amdgcn_alignbit(a, b, 32 - sh) : a;
    };
    const uint32_t a = dense[q0], b = dense[q0 + 1];
    const uint32_t la = dense[q + nmid], lb = dense[q + nmid + 1];
    uint32_t cur = dense[q];
    uint32_t n1 = dense[q + 1], n2 = dense[q + 2], n3 = dense[q + 3],
             n4 = dense[q + 4];
    {
        uint32_t v = os ? __builtin_amdgcn_alignbit(a, b, 32 - os) : a;
        v >>= od;
        if (w0 == wl)
            v &= tailm;
        __hip_atomic_fetch_or(&st[w0], bswap32(v), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (wl == w0)
        return;
    QH_LDS uint32_t *o = st + w0 + 1;
    // (!Mid: the whole wave copies the middle words, copy_dense_mid)
    for (uint32_t k = 0; k < (Mid ? nmid : 0u); k += 4)
    {
        if (k)
        {
            n1 = dense[q + k + 1];
            n2 = dense[q + k + 2];
            n3 = dense[q + k + 3];
            n4 = dense[q + k + 4];
        }
        o[k] = bswap32(win(cur, n1));
        if (k + 1 < nmid)
            o[k + 1] = bswap32(win(n1, n2));
        if (k + 2 < nmid)
            o[k + 2] = bswap32(win(n2, n3));
        if (k + 3 < nmid)
            o[k + 3] = bswap32(win(n3, n4));
        cur = n4;
    }
    __hip_atomic_fetch_or(&st[wl], bswap32(win(la, lb) & tailm),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the words a string of nb dense bits from bit s to the byte-aligned bit d
// owns whole (copy_dense<false> leaves them), by the whole wave
__device__ __forceinline__ void
copy_dense_mid(const QH_LDS uint32_t *dense, uint32_t s, uint32_t nb,
               QH_LDS uint32_t *st, uint32_t d)
{
    const uint32_t w0 = d >> 5, wl = (d + nb - 1) >> 5;
    const uint32_t nmid = wl > w0 ? wl - w0 - 1 : 0u;
    const uint32_t x1 = s - (d & 31) + 32, sh = x1 & 31, q = x1 >> 5;
    QH_LDS uint32_t *o = st + w0 + 1;
    for (uint32_t k = lane_id(); k < nmid; k += 64)
    {
        const uint32_t a = dense[q + k], b = dense[q + k + 1];
        o[k] = bswap32(sh ? __builtin_amdgcn_alignbit(a, b, 32 - sh) : a);
    }
}

// Huffman payloads of more dense bits than this are copied by the whole
// wave (a lane alone copies 4 words a trip: a 1 KB value would take ~60
// trips while the others idle)
#ifndef QH_ENC_COOP_BITS
#define QH_ENC_COOP_BITS 1024
#endif
#ifndef QH_ENC_COOP                          // 0: every payload by its lane
#define QH_ENC_COOP 1
#endif
constexpr uint32_t kEncCoopBits = QH_ENC_COOP_BITS;

// one string from the dense stream: framing, payload bits [s, s + bits),
// padding; raw strings (E3 fallback) from the staged input.  Returns the
// payload's first bit.
__device__ __forceinline__ uint32_t
emit_dense(const QH_LDS uint32_t *in, uint32_t rs, uint32_t re, uint32_t mode,
           const EncSize &z, const QH_LDS uint32_t *dense, uint32_t s,
           uint32_t bits, const QH_LDS u32x2 *s_enc, QH_LDS uint32_t *st,
           uint32_t start)
{
    uint32_t pos = 8 * start;
    if (mode)
        pos = emit_prefix(st, pos, mode, z.huff, z.plen);
    const uint32_t p0 = pos;
    if (!z.huff)
    {
        pack_bits(in, rs, re, true, s_enc, st, pos);
        return p0;
    }
    if (bits)
    {
        copy_dense(dense, s, bits, st, pos);
        pos += bits;
        const uint32_t pad = (8 - (pos & 7)) & 7;
        if (pad)
            or_bits(st, pos, (1u << pad) - 1, pad);
    }
    return p0;
}

// A tile whose input or output does not fit the stages, coded eagerly:
// sizes from the stage (given) or from global memory, then packed straight
// to global memory.  The tile's output base comes from base_of(total) (the
// batch kernel's look-back, or the service's running offset); its offsets go
// to t_off (the tile's first string).  Returns base + total.  Out of line
// (cold), state by value.
template <class SM, class BaseOf>
__device__ __noinline__ uint64_t
enc_slow_tile(const uint8_t *in, uint32_t mode, QH_LDS SM *sm,
              QH_LDS EncWave *wv, uint32_t rs, uint32_t re, EncSize z,
              uint32_t cnt, TileOffs to, Span sp, uint32_t sz, bool sized,
              uint8_t *out, uint32_t *t_off, BaseOf base_of)
{
    const uint32_t lane = lane_id();
    const bool valid = lane < cnt;
    const EncGlb gsrc{(const QH_GLB uint32_t *) sp.pa};
    if (!sp.staged)
    {
        rs = valid ? (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa) : 0;
        re = valid ? (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa) : 0;
        if (!sized)
        {
            z = (EncSize){0, 0, true};
            if (valid)
                z = size_string(mode, gsrc, rs, re, sm->len);
            sz = z.size;
        }
    }
    const uint32_t incl = wave_incl_scan(sz);
    const uint32_t excl = incl - sz;
    const uint32_t total = read_lane(incl, 63);
    const uint64_t base = base_of(total);
    if (valid && sz)
    {
        const uint32_t adj = (uint32_t) ((uintptr_t) out & 3);
        Packer<PackGlb> pk;
        pk.sink.out = out - adj;
        const uint32_t p0 = adj + (uint32_t) base + excl;
        pk.init(p0, p0 + sz);
        if (sp.staged)
            emit_string(EncLds{wv->in}, rs, re, mode, z.huff, z.plen, sm->enc,
                        pk);
        else
            emit_string(gsrc, rs, re, mode, z.huff, z.plen, sm->enc, pk);
    }
    if (valid)
        ((QH_GLB uint32_t *) t_off)[lane] = (uint32_t) (base + excl);
    return base + total;
}


// the sizes of a tile past the stage, from global memory (as enc_slow_tile
// sizes them with sized = false)
template <class SM>
__device__ __noinline__ EncSize
enc_tile_sizes(const uint8_t *in, uint32_t mode, QH_LDS SM *sm, uint32_t cnt,
               TileOffs to, Span sp)
{
    EncSize z = (EncSize){0, 0, true};
    if (lane_id() < cnt)
    {
        const EncGlb gsrc{(const QH_GLB uint32_t *) sp.pa};
        const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa);
        const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa);
        z = size_string(mode, gsrc, rs, re, sm->len);
    }
    return z;
}

template <class SM>
__device__ __forceinline__ bool
enc_big_sizes(const uint8_t *in, uint32_t mode, QH_LDS SM *sm,
              QH_LDS EncWave *wv, uint32_t cnt, TileOffs to, Span sp,
              uint32_t &sz, uint8_t *dst);

// the encode side of the wave pipeline (qhuff_pipeline.h, qhuff_service.hip);
// SM: the workgroup's LDS (enc, mt, len)
template <class SM, bool Full = true>
struct EncPolicyT
{
    static constexpr bool kStatus = false;
    // Full: big tiles through output slots, long payloads copied by the
    // wave (see DecPolicyT)
    static constexpr bool kBig = Full;
    static constexpr bool kCoop = false;          // (no coop_phase)
    static constexpr uint64_t coop = 0;
    static constexpr int kInCap = kEncInCap;
    static constexpr int kDepth = QH_ENC_DEPTH;       // pending tiles
    static constexpr int kOutCap = kEncOutCap;
    static constexpr int kNch = kChunks;          // 16-byte chunks per lane
    static constexpr uint32_t kTS = kWT;          // strings per tile
    using Offs = TileOffs;
    const uint8_t *in;
    uint32_t mode;                   // 0 payload, 3/5/7 literal prefix bits
    QH_LDS SM *sm;
    QH_LDS EncWave *wv;
    uint32_t rs, re;                 // this lane's string in the stage
    uint32_t ds, bits;               // its range of the dense stream
    EncSize z;
    uint32_t dense;                  // wave-uniform: tile from the dense stream

    // staged tile: chunks into the LDS stage
    __device__ __forceinline__ void stage_in(const Chunks<kChunks> &ch,
                                             const Span &sp, const TileOffs &)
    {
        ch.store<false>((QH_LDS u32x4 *) wv->in, sp.n16);
    }
    // the byte-parallel pass over the stage (after the next tile's loads
    // have been issued into the chunk registers)
    __device__ __forceinline__ void prepare(const Span &sp)
    {
        if constexpr (SM::kMtRep)
            dense_pass<true>(sp.n16, sm->mtr, wv);
        else
            dense_pass<false>(sp.n16, sm->mt, wv);
        dense = true;
    }
    __device__ __forceinline__ const QH_LDS uint32_t *out_stage() const
    {
        return wv->out;
    }
    // staged tile: size this lane's string (E1, and the E3 choice)
    __device__ __forceinline__ void codec(const TileOffs &to, uint32_t cnt,
                                          const Span &sp, uint32_t *sz,
                                          uint32_t *st)
    {
        codec_range(to, 0, cnt, sp, sz, st);
    }
    __device__ __forceinline__ void coop_phase(const TileOffs &, uint32_t,
                                               uint32_t, const Span &,
                                               uint32_t *, uint32_t *)
    {
    }
    // the strings of lanes [lo, cnt) (sp: their span, prepared)
    __device__ __forceinline__ void codec_range(const TileOffs &to, uint32_t lo,
                                                uint32_t cnt, const Span &sp,
                                                uint32_t *sz, uint32_t *st)
    {
        const uint32_t lane = lane_id();
        const bool valid = (lane >= lo) & (lane < cnt);
        rs = valid ? (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa) : 0;
        re = valid ? (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa) : 0;
        z = (EncSize){0, 0, true};
        if (dense)
        {
            // string i spans the dense bits between the offsets of its ends
            const uint32_t se = dense_at(wv, re);
            const uint32_t ra = (uint32_t) ((uintptr_t) (in + read_lane(to.o0, lo))
                                            - sp.pa);
            const uint32_t s_first = dense_at(wv, ra);
            uint32_t prev = wave_shr1(se);
            // (every lane shifts: not moved into the select's branch)
            asm volatile("" : "+v"(prev));
            ds = lane != lo ? prev : s_first;
            bits = se - ds;
            dense = read_lane(se, cnt - 1) + 64 <= kDenseBits;
        }
        if (valid)
            z = dense ? size_from_bits(mode, bits, re - rs)
                      : size_string(mode, EncLds{wv->in}, rs, re, sm->len);
        *sz = z.size;
        *st = 0;
    }
    // pack (E2 / E3) into the zeroed output stage
    __device__ __forceinline__ void emit(uint32_t excl, uint32_t sz,
                                         uint32_t total)
    {
        QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) wv->out;
        const uint32_t n16 = (total + 15) / 16 + 1;
        for (uint32_t i = lane_id(); i < n16; i += 64)
            o4[i] = (u32x4){0, 0, 0, 0};
        wave_sync();
#ifdef QH_TIME_NO_EMIT                       // timing builds only: no output
        return;
#endif
        if (dense)
        {
            // long payloads: their middle words by the whole wave, after
            const bool lc = Full && QH_ENC_COOP && (sz != 0) & z.huff
                          & (bits > kEncCoopBits);
            const uint64_t lm = __builtin_amdgcn_ballot_w64(lc);
            uint32_t p0 = 0;
            if (sz)
                p0 = emit_dense(wv->in, rs, re, mode, z, wv->dense, ds,
                                lc ? 0u : bits, sm->enc, wv->out, excl);
            if (lm)
            {
                if (lc)
                {
                    // its first and last words (shared), and the padding
                    copy_dense<false>(wv->dense, ds, bits, wv->out, p0);
                    const uint32_t pe = p0 + bits;
                    const uint32_t pad = (8 - (pe & 7)) & 7;
                    if (pad)
                        or_bits(wv->out, pe, (1u << pad) - 1, pad);
                }
                uint64_t m = lm;
                while (m)
                {
                    const uint32_t j = (uint32_t) __builtin_ctzll(m);
                    m &= m - 1;
                    copy_dense_mid(wv->dense, read_lane(ds, j),
                                   read_lane(bits, j), wv->out,
                                   read_lane(p0, j));
                }
            }
        }
        else if (sz)
            emit_bits(wv->in, rs, re, mode, z.huff, z.plen, sm->enc, wv->out,
                      excl);
    }

    // a tile of the batch kernel: base from the look-back
    // a big tile's sizes, and its output into dst when it fits
    __device__ __forceinline__ bool big_sizes(uint32_t cnt, TileOffs to, Span sp,
                                              uint32_t &sz, uint32_t &st,
                                              uint8_t *dst)
    {
        st = 0;
        return enc_big_sizes(in, mode, sm, wv, cnt, to, sp, sz, dst);
    }
    // a big tile whose output does not fit a slot (qhuff_pipeline.h), after
    // the pending tiles are flushed: base from the look-back
    // the sizes of a tile past the stage (the lean kernel: no codec ran)
    __device__ __forceinline__ void slow_size(uint32_t cnt, TileOffs to, Span sp,
                                              uint32_t &sz, uint32_t &st)
    {
        z = enc_tile_sizes(in, mode, sm, cnt, to, sp);
        sz = z.size;
        st = 0;
    }
    // ... its output once the look-back lb (aggregate published) resolves
    __device__ __forceinline__ void slow_tile(Coord c, uint32_t t, uint32_t cnt,
                                              TileOffs to, Span sp, uint32_t sz,
                                              uint32_t, bool sized, uint8_t *out,
                                              uint32_t *out_off, uint8_t *,
                                              uint64_t n, const LookBack &lb)
    {
        // sized: z from slow_size (the lean kernel) -- a full kernel's big
        // tile has its sizes from big_sizes but not z, so it sizes again
        const uint64_t end = enc_slow_tile(in, mode, sm, wv, rs, re, z, cnt,
                                              to, sp, sz, sized, out,
                                              out_off + (uint64_t) t * kTS,
                                              StartedBase{c, lb});
        last_tile_end(c, t, end, out_off, n);
    }
    // a tile at a known base
    __device__ __forceinline__ uint64_t slow_tile_at(uint64_t base, uint32_t cnt,
                                                     TileOffs to, Span sp,
                                                     uint32_t sz, uint32_t,
                                                     uint8_t *out, uint32_t *t_off,
                                                     uint8_t *)
    {
        return enc_slow_tile(in, mode, sm, wv, rs, re, z, cnt, to, sp, sz, false,
                                out, t_off, FixedBase{base});
    }
};


// The sizes of a big tile and, when they fit kBigSlotBytes, its whole
// packed output at dst (a big-tile slot, qhuff_pipeline.h), written before
// its base is known.  Staged input (sizes given by the main codec): packed
// by each lane from the stage.  Otherwise unit by unit, each staged,
// dense-passed, sized and packed into the out stage (or, past it, by each
// lane); a string whose input alone exceeds the stage is sized and packed
// from global memory by its lane.  Returns whether all of the output went to
// dst; the sizes are complete either way.
template <class SM>
__device__ __forceinline__ bool
enc_big_sizes(const uint8_t *in, uint32_t mode, QH_LDS SM *sm,
              QH_LDS EncWave *wv, uint32_t cnt, TileOffs to, Span sp,
              uint32_t &sz, uint8_t *dst)
{
    using P = EncPolicyT<SM, true>;
    P pol{in, mode, sm, wv};
    const uint32_t lane = lane_id();
    const bool valid = lane < cnt;
    // per-lane packing of lanes [lo, hi) from the LDS stage (span su) at
    // dst + at (this lane's offset)
    auto pack_lds = [&](uint32_t lo, uint32_t hi, const Span &su, uint32_t at) {
        if ((lane >= lo) & (lane < hi))
        {
            const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - su.pa);
            const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - su.pa);
            const EncSize z = size_string(mode, EncLds{wv->in}, rs, re, sm->len);
            if (z.size)
            {
                Packer<PackGlb> pk;
                pk.sink.out = dst;
                pk.init(at, at + z.size);
                emit_string(EncLds{wv->in}, rs, re, mode, z.huff, z.plen,
                            sm->enc, pk);
            }
        }
    };
    if (sp.staged)
    {
        const uint32_t s = valid ? sz : 0u;
        const uint32_t incl = all_lanes(wave_incl_scan(s));
        if (read_lane(incl, 63) > kBigSlotBytes)
            return false;
        pack_lds(0, cnt, sp, incl - s);
        return true;
    }
    uint32_t run = 0;
    bool fits = true;
    sz = 0;
    for (uint32_t i0 = 0; i0 < cnt;)
    {
        const uint32_t k = unit_len(in, to, i0, cnt, P::kInCap, false, 0, 0, 0);
        if (k == 0)
        {
            // one string beyond the stage, from global memory by its lane
            const uintptr_t pa = (uintptr_t) (in + read_lane(to.o0, i0))
                               & ~(uintptr_t) 15;
            const EncGlb src{(const QH_GLB uint32_t *) pa};
            const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - pa);
            const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - pa);
            EncSize z = (EncSize){0, 0, true};
            if (lane == i0)
            {
                z = size_string(mode, src, rs, re, sm->len);
                sz = z.size;
            }
            const uint32_t n = read_lane(sz, i0);
            fits = fits && run + n <= kBigSlotBytes;
            if (fits && lane == i0 && n)
            {
                Packer<PackGlb> pk;
                pk.sink.out = dst;
                pk.init(run, run + n);
                emit_string(src, rs, re, mode, z.huff, z.plen, sm->enc, pk);
            }
            run += n;
            i0 += 1;
            continue;
        }
        const uint32_t i1 = i0 + k;
        const Span su = tile_span(in, read_lane(to.o0, i0),
                                  read_lane(to.o1, i1 - 1), P::kInCap);
        stage_chunks<false>(su, (QH_LDS u32x4 *) wv->in);
        pol.prepare(su);
        wave_sync();
        uint32_t s1, t1;
        pol.codec_range(to, i0, i1, su, &s1, &t1);
        const bool in_u = (lane >= i0) & (lane < i1);
        const uint32_t ls = in_u ? s1 : 0u;
        const uint32_t incl = all_lanes(wave_incl_scan(ls));
        const uint32_t ut = read_lane(incl, 63);
        fits = fits && run + ut <= kBigSlotBytes;
        if (fits)
        {
            if (ut + 64 <= (uint32_t) P::kOutCap)
            {
                wave_sync();
                pol.emit(in_u ? incl - ls : 0u, ls, ut);
                wave_sync();
                copy_out((const QH_LDS uint8_t *) wv->out, dst + run, ut);
            }
            else
                pack_lds(i0, i1, su, run + incl - ls);
        }
        if (in_u)
            sz = s1;
        run += ut;
        wave_sync();
        i0 = i1;
    }
    return fits;
}

// the code tables, loaded once per workgroup (threads 0..256)
template <class SM>
__device__ __forceinline__ void
enc_tables_load(QH_LDS SM *sm, const uint2 *enc_g, int tid)
{
    const QH_GLB u32x2 *genc = (const QH_GLB u32x2 *) enc_g;
    if (tid < 257)
    {
        const u32x2 e = genc[tid];
        sm->enc[tid] = e;
        if (tid < 256)
        {
            sm->len[tid] = (uint8_t) e.y;
            // (codes of 28 and 30 bits keep their low 27: the bits above
            // are ones, dense_pass puts them back)
            const uint32_t m = mt_entry(e.x, e.y);
            sm->mt[tid] = m;
            if constexpr (SM::kMtRep)
            {
                QH_LDS u32x4 *r = (QH_LDS u32x4 *) &sm->mtr[tid * 32];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    r[k] = (u32x4){m, m, m, m};
            }
        }
    }
}

}  // namespace qhuff
