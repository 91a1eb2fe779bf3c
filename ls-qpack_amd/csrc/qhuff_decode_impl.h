// qhuff_decode_impl.h -- the decode side of the kernels: window-table
// step loop, arena compaction, slow tiles and the tile policy, shared by the
// batch kernel (qhuff_decode.hip) and the service kernel (qhuff_service.hip).
// See qhuff_decode.hip for the algorithm.
#pragma once

#include "qhuff_pipeline.h"

#ifndef QH_DEPTH
#define QH_DEPTH 3
#endif
// bytes past the last slot's bound (the two-byte emitter writes one past
// its end)
#ifndef QH_ARENA_SLACK
#define QH_ARENA_SLACK 16
#endif

namespace qhuff {


// window entry fields (qhuff_tables.h)
__device__ __forceinline__ uint32_t ent_c(uint32_t e) { return (e >> 8) & 15; }
__device__ __forceinline__ uint32_t ent_l0(uint32_t e) { return (e >> 12) & 15; }
__device__ __forceinline__ uint32_t ent_ns(uint32_t e) { return (e >> 24) & 3; }
__device__ __forceinline__ uint32_t ent_sym1(uint32_t e) { return (e >> 16) & 0xff; }

// staged input bytes (the output stage, the dead input stage, always has the
// chunk registers' 3,072); a smaller cap lets more waves fit the LDS (16
// waves at 2,816 B were slower: dec 88 vs 86 us, round 1)
constexpr int kDecNch = kChunks;                        // chunks per lane
constexpr uint32_t kDecTS = kWT;                        // strings per tile
constexpr int kDecStageCap = 64 * kDecNch * 16;
#ifndef QH_DEC_IN_CAP
#define QH_DEC_IN_CAP 3072
#endif
constexpr int kDecInCap = QH_DEC_IN_CAP;
static_assert(kDecInCap % 16 == 0 && kDecInCap <= kDecStageCap, "input cap");
// byte slot of string i: 2i + floor(8 * (rs_i - A) / 5) -- an output is at
// most 8/5 of its input, plus one byte written past the end by the
// two-byte emitter
constexpr int kVarArenaBytes = 2 * kDecTS + 8 * kDecInCap / 5 + QH_ARENA_SLACK;
// Tiles whose strings are all short enough use a fixed-stride arena
// instead: lane l's slot at kFixStride * l.  The stride is an odd number of
// dwords, so the byte stores of lanes that have emitted about as many
// bytes fall on distinct banks (with slots placed by input offset the 64
// stores of a step land on random banks: the stores were two thirds of the
// step loop's LDS bank-conflict cycles, profiles/r03_b).  A string of at
// most kFixMaxLen Huffman bytes decodes to at most floor(8 * len / 5) bytes
// and the emitter writes one past its end.
#ifndef QH_FIX_STRIDE
#define QH_FIX_STRIDE 108
#endif
constexpr uint32_t kFixStride = QH_FIX_STRIDE;
static_assert(kFixStride % 8 == 4, "an odd number of dwords");
constexpr uint32_t kFixMaxLen = (5 * (kFixStride - 1)) / 8;
constexpr int kArenaBytes = kVarArenaBytes > (int) (64 * kFixStride)
                          ? kVarArenaBytes : (int) (64 * kFixStride);

struct DecWave                       // one wave's private LDS region
{
    alignas(16) uint32_t in[kDecStageCap / 4];   // BE input dwords; output stage
    alignas(16) uint8_t arena[kArenaBytes];
};

// hold entry, one past the window table: c = 0, ns = 0, not a long code
constexpr uint32_t kHoldIdx = kWinSize;
constexpr uint32_t kHoldEntry = 1u << 26;

struct DecSmem
{
    uint32_t win[kWinSize + 4];      // + the hold entry
    uint16_t sorted[257];
    uint16_t long2[kLong2Size];      // long codes by leading ones
    DecWave w[kWaves];
    BlockTickets tk;                 // the workgroup's first tickets
};

struct DecLds                        // big-endian dwords staged in LDS
{
    const QH_LDS uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
    // the stage has slack past the input: reading ahead is always safe
    __device__ __forceinline__ uint32_t dw_ahead(uint32_t i, uint32_t) const
    {
        return w[i];
    }
};
struct DecGlb                        // raw little-endian bytes in global
{
    const QH_GLB uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const
    {
        return bswap32(w[i]);
    }
    // never touch a dword that holds no byte of the string (page safety)
    __device__ __forceinline__ uint32_t dw_ahead(uint32_t i,
                                                 uint32_t bitend) const
    {
        return i * 32 < bitend ? bswap32(w[i]) : 0u;
    }
};

// long-code step: canonical search over the code lengths 13..30 (compile-
// time parameters, one compare-and-select per length)
template <int I>
__device__ __forceinline__ void
long_search(uint32_t w, uint32_t &L, uint32_t &idx)
{
    if constexpr (I < (int) kLongTab.n)
    {
        constexpr LongLen ll = kLongTab.l[I];
        const uint32_t off = (w >> (32 - ll.len)) - ll.first;
        const bool hit = (L == 0) & (off < ll.count);
        L = hit ? ll.len : L;
        idx = hit ? ll.base + off : idx;
        long_search<I + 1>(w, L, idx);
    }
}

__device__ __forceinline__ uint32_t
long_code(uint32_t w, const QH_LDS uint16_t *s_sorted, uint32_t *len)
{
    uint32_t L = 0, idx = 0;
    long_search<0>(w, L, idx);
    *len = L;
    return s_sorted[idx];
}

// One main-phase step: look the top 12 bits up, emit up to two symbols,
// shift them out of the 64-bit buffer hi:lo and refill one dword when fewer
// than 32 valid bits remain.  GATED: lanes with act == false keep their
// state (consume 0 bits, emit 0 bytes).  Returns false for a lane that hit
// the EOS code (the string is rejected, D3 (a)).
template <bool GATED, class Emit>
__device__ __forceinline__ bool
main_step(bool act, uint32_t d, uint32_t &hi, uint32_t &lo, uint32_t &bits,
          uint32_t &rem, uint32_t &p, const QH_LDS uint32_t *s_win,
          const QH_LDS uint16_t *s_sorted, Emit &emit)
{
    uint32_t e = s_win[hi >> (32 - kWinBits)];
    bool ok = true;
    if (__builtin_amdgcn_ballot_w64((GATED ? act : true) & (e < (1u << 24))))
    {
        // a code of 13..30 bits: synthesize the entry of a one-symbol step
        uint32_t L;
        const uint32_t sym = long_code(hi, s_sorted, &L);
        const bool lng = (GATED ? act : true) & (e < (1u << 24));
        ok = !(lng & (sym == 256));
        const uint32_t el = (sym & 0xff) | (L << 8) | (L << 12) | (1u << 24)
                          | ((32u - L) << 26);
        e = lng ? (ok ? el : 0u) : e;
    }
    if (GATED)
        e = act ? e : 0u;
    const uint32_t nb = (e >> 24) & 3;       // 0 for a held lane
    const uint32_t k = e >> 26;              // 32 - bits consumed
    const uint32_t cc = 32u - k;
    emit(e, nb);
    const uint32_t sh = __builtin_amdgcn_alignbit(hi, lo, k);
    hi = GATED ? (nb ? sh : hi) : sh;
    lo = lo << (cc & 31);                    // held: cc = 32, no shift
    const uint32_t used = GATED ? (nb ? cc : 0u) : cc;
    bits -= used;
    rem -= used;
    const bool need = bits < 32;
    const uint32_t dd = need ? d : 0u;
    hi |= dd >> (bits & 31);
    lo |= dd << ((32 - bits) & 31);
    p += need ? 1 : 0;
    bits += need ? 32 : 0;
    return ok;
}

// Decode one string whose bits are [bit0, bitend) of the big-endian dword
// stream `src`; emitted bytes go through `emit`.  Returns the number of
// output bytes, or -1 - k for a rejected string (k: the bytes emitted before
// the error, every symbol before the EOS code or before the bad padding).
// Three wave-uniform phases:
//   1. while every lane has >= 32 real bits ahead: ungated steps;
//   2. while some lane does: steps predicated on the lane's own state;
//   3. the last < 32 bits, padded with ones, with the D3 tail rule.
template <class Src, class Emit>
__device__ __forceinline__ int
decode_string(const Src &src, uint32_t bit0, uint32_t bitend,
              const QH_LDS uint32_t *s_win, const QH_LDS uint16_t *s_sorted,
              Emit &emit)
{
    uint32_t rem = bitend - bit0;            // real bits not yet consumed
    uint32_t hi = 0, lo = 0, bits = 0, p = 0;
    if (rem)
    {
        const uint32_t i0 = bit0 >> 5, sk = bit0 & 31;
        const uint32_t a = src.dw(i0), b = src.dw_ahead(i0 + 1, bitend);
        hi = sk ? __builtin_amdgcn_alignbit(a, b, 32 - sk) : a;
        lo = b << sk;
        bits = 64 - sk;
        p = i0 + 2;
    }
    bool bad = false;

    // Invariant in phases 1-2: the buffer holds >= 32 valid bits and ends
    // on a dword boundary (p).  A held lane's two arena byte writes land at
    // its current end and are overwritten or ignored.
    if (!__builtin_amdgcn_ballot_w64(rem < 32))
    do
    {
        const uint32_t d = src.dw_ahead(p, bitend);
        const bool ok = main_step<false>(true, d, hi, lo, bits, rem, p, s_win,
                                         s_sorted, emit);
        bad |= !ok;
        rem = ok ? rem : 0u;                 // leave phase 1 (rare)
    } while (!__builtin_amdgcn_ballot_w64(rem < 32));
    bool act = rem >= 32 && !bad;
    if (__builtin_amdgcn_ballot_w64(act))
    do
    {
        const uint32_t d = src.dw_ahead(p, bitend);
        const bool ok = main_step<true>(act, d, hi, lo, bits, rem, p, s_win,
                                        s_sorted, emit);
        bad |= !ok;
        act = act & ok & (rem >= 32);
    } while (__builtin_amdgcn_ballot_w64(act));

    // epilogue: the last < 32 bits, padded with ones; D3 tail rule
    bool fin = bad || rem == 0;
    if (__builtin_amdgcn_ballot_w64(!fin))
    do
    {
        const uint32_t w = hi | (0xffffffffu >> (rem & 31));
        const uint32_t e = s_win[w >> (32 - kWinBits)];
        const uint32_t ns = ent_ns(e), ct = ent_c(e), l0 = ent_l0(e);
        const bool two = (ns == 2) & (ct <= rem);
        uint32_t c = two ? ct : (ns ? l0 : 31u);
        uint32_t val = e;
        bool eos = false;
        if (__builtin_amdgcn_ballot_w64(!fin & (ns == 0) & (rem > kWinBits)))
        {
            uint32_t L;
            const uint32_t sym = long_code(w, s_sorted, &L);
            const bool lng = (ns == 0) & (rem > kWinBits);
            c = lng ? L : c;
            val = lng ? sym : val;
            eos = lng & (sym == 256);
        }
        // c > rem: what is left is padding -- at most 7 bits of EOS prefix
        const bool over = c > rem;
        const uint32_t ones = 0xffffffffu >> ((32 - rem) & 31);
        const bool tail_bad = rem >= 8 || (w >> ((32 - rem) & 31)) != ones;
        const bool live = !fin;
        bad |= live & ((over & tail_bad) | (!over & eos));
        const bool step = live & !over & !eos;
        const uint32_t nb = step ? (two ? 2u : 1u) : 0u;
        c = step ? c : 0;
        emit(val, nb);
        const uint32_t sh = __builtin_amdgcn_alignbit(hi, lo, (32 - c) & 31);
        hi = c ? sh : hi;
        lo = lo << (c & 31);
        rem -= c;
        fin = fin | over | eos | (rem == 0);
    } while (__builtin_amdgcn_ballot_w64(!fin));
    return bad ? -1 - (int) emit.n : (int) emit.n;
}

// Lean variant used by the staged (LDS) path (same return value).  The bit stream sits in two
// dwords A:B with a position t: the 32-bit window is alignbit(A, B, t) --
// ((A:B) >> t), the next bit at A's bit 31 - (32 - t) -- valid for t in
// [0, 31] (t = 0: the window is B).  Consuming c bits lowers t; when it goes
// negative the window moves on a dword (A = B, B = the next dword, read one
// step ahead) and t wraps (t & 31).  No 64-bit shifts, and the window always
// holds 32 stream bits, enough for any code.  Main steps run while a lane
// has at least kWinBits real bits left, so the window's top kWinBits bits
// hold no padding and every symbol of its entry is real (a lane past that
// reads the hold entry: it consumes and emits nothing); the EOS check and
// the "code runs past the end" check (the leftover would be >= 8 bits: D3)
// live in the rare long-code branch.  The last < kWinBits bits (at most two
// symbols) take the padded epilogue with the D3 tail rule, exactly as
// decode_string().
// R2: two main steps per loop trip share one refill read of the next input
// dword (step lab at 12 waves/CU: 8,633 vs 9,795 cycles per tile; decode
// 62.7 vs 64.0 us in-process, profiles/r03_p); false: one read per step.
template <class Emit, bool R2 = true>
__device__ __forceinline__ int
decode_string_lds(const QH_LDS uint32_t *src, uint32_t bit0, uint32_t bitend,
                  const QH_LDS uint32_t *s_win, const QH_LDS uint16_t *s_sorted,
                  const QH_LDS uint16_t *s_long2, Emit &emit)
{
    uint32_t rem = bitend - bit0;            // real bits not yet consumed
    uint32_t A, B, t, p, nx;
    {
        const uint32_t i0 = bit0 >> 5, sk = bit0 & 31;
        A = src[i0];
        const uint32_t a1 = src[i0 + 1];
        B = sk ? a1 : A;                     // sk == 0: the window is B = A
        t = (32 - sk) & 31;
        p = sk ? i0 + 2 : i0 + 1;
        nx = src[p];
    }
    uint32_t bad = 0;                        // (a u32: no lane-mask phis)
    // No lane branches in the step: a lane with < kWinBits real bits left
    // looks up the hold entry (c = ns = 0, never a long code); its two arena
    // byte writes land at its current end and are overwritten by the
    // epilogue.
    constexpr uint32_t kMain = kWinBits;
    uint32_t W = __builtin_amdgcn_alignbit(A, B, t);
    // idx is the entry's byte offset: (W >> 17) & 0x7ffc for a live lane,
    // the hold entry's for a held one -- one v_and_or on the step's chain
    // (the two masks come off the rem compare, beside it).  (One select
    // after the masked shift, a VALU fewer but one longer on the chain, was
    // neutral: dec 66.16 vs 66.21 us, profiles/r02_r/ab_addr2.txt.)
    auto win_addr = [](uint32_t w, bool live) -> uint32_t {
        return ((w >> (32 - kWinBits - 2)) & (live ? 4u * (kWinSize - 1) : 0u))
             | (live ? 0u : 4u * kHoldIdx);
    };
    uint32_t idx = win_addr(W, rem >= kMain);
    // A long-code marker entry (e < 2^24: c = ns = 0, no bytes) stalls its
    // lane where it is, like the hold entry, for the rest of the loop trip;
    // at the trip's end, if any lane is stalled, the stalled lanes take
    // their long step at once (one count of leading ones, one long2 lookup),
    // the others wait that one step.  (Until round 4 the stalled lanes
    // waited until every live lane was stalled or done: on text with ~2 %
    // long-code bytes a wave then ran its step count about twice,
    // alphabet C decoded at 1.9x the token batch's time.)  The token
    // batch's step is unchanged: one more scalar test per trip.
    auto advance = [&](uint32_t c) {
        uint32_t tn;
        const bool cross = __builtin_sub_overflow(t, c, &tn);
        A = cross ? B : A;
        B = cross ? nx : B;
        t = tn & 31;
        p += cross ? 1u : 0u;
    };
    if (__builtin_amdgcn_ballot_w64(rem >= kMain))
    do
    {
        uint32_t e = *(const QH_LDS uint32_t *) ((const QH_LDS uint8_t *) s_win + idx);
        const uint32_t c = ent_c(e);
        emit(e, ent_ns(e));
        rem -= c;
        advance(c);
        if constexpr (!R2)
            nx = src[p];
        W = __builtin_amdgcn_alignbit(A, B, t);
        idx = win_addr(W, rem >= kMain);
        if constexpr (R2)
        {
            // A second step on the same refill: a main step consumes at
            // most 13 bits, and a step that moves the window on a dword
            // leaves t >= 19, so the two steps cross at most one dword
            // boundary and the next dword nx read before them covers it.
            // (A lane that stalled or went on hold in the first step
            // reads the same entry again and consumes nothing.)
            e = *(const QH_LDS uint32_t *) ((const QH_LDS uint8_t *) s_win + idx);
            const uint32_t c2 = ent_c(e);
            emit(e, ent_ns(e));
            rem -= c2;
            advance(c2);
            nx = src[p];
            W = __builtin_amdgcn_alignbit(A, B, t);
            idx = win_addr(W, rem >= kMain);
        }
        // lanes with >= kMain bits on a marker sit on a code of 14..30
        // bits; EOS, or a code running past the end, rejects the string (D3)
        const bool lng = (rem >= kMain) & (e < (1u << 24));
        if (__builtin_expect(__builtin_amdgcn_ballot_w64(lng) != 0, 0))
        {
            // (a long step consumes at most 30 bits: it crosses at most one
            // dword, which nx holds)
            const uint32_t n1 = min(~W ? (uint32_t) __builtin_clz(~W) : 32u,
                                    31u);
            const uint32_t x = (W << ((n1 + 1) & 31)) >> 27;
            const uint32_t l2 = s_long2[(lng ? n1 - kLong2N1 : 0u) * 32 + x];
            const uint32_t sym = l2 & 511, L = (l2 >> 9) + 14;
            const bool rej = lng & ((sym == 256) | (L > rem));
            const bool ok = lng & !rej;
            const uint32_t cl = ok ? L : 0u;
            emit(sym, ok ? 1u : 0u);
            bad |= rej ? 1u : 0u;
            rem = rej ? 0u : rem - cl;
            advance(cl);
            nx = src[p];
            W = __builtin_amdgcn_alignbit(A, B, t);
            idx = win_addr(W, rem >= kMain);
        }
    } while (__builtin_amdgcn_ballot_w64(rem >= kMain));

    // epilogue, one pass: the last < kWinBits (13) real bits hold at most
    // two symbols (codes are >= 5 bits), both inside the window padded with
    // ones, so one lookup decodes them; the bits after them cannot complete
    // a code (its entry would have decoded it), so they are the padding, and
    // the D3 tail rule (fewer than 8 bits, all ones) applies at once.  The
    // EOS code (30 bits) cannot occur in 12 bits.
    {
        const bool live = !(bad || rem == 0);
        const uint32_t w = W | (0xffffffffu >> (rem & 31));
        const uint32_t e = s_win[w >> (32 - kWinBits)];
        const uint32_t ns = ent_ns(e), ct = ent_c(e), l0 = ent_l0(e);
        const bool two = (ns == 2) & (ct <= rem);
        const bool one = !two & (ns != 0) & (l0 <= rem);
        const uint32_t c = two ? ct : (one ? l0 : 0u);
        emit(e, live ? (two ? 2u : (one ? 1u : 0u)) : 0u);
        const uint32_t r2 = rem - c;             // padding bits
        const uint32_t inv = ~(w << (c & 31));   // padding bits at the top
        const bool pad_ok = r2 < 8 && (r2 == 0 || (inv >> ((32 - r2) & 31)) == 0);
        bad |= (live & !pad_ok) ? 1u : 0u;
    }
    emit.finish();
    return bad ? -1 - (int) emit.n : (int) emit.n;
}

// byte-granular arena sink: two unconditional byte stores per step, the
// entry's first symbol [7:0] and second [23:16] (ds_write_b8 / _d16_hi; the
// second is overwritten by the next step when only one symbol was emitted)
struct ArenaEmit
{
    QH_LDS uint8_t *slot;
    QH_LDS uint8_t *p;
    uint32_t n;
    __device__ __forceinline__ void finish() { n = (uint32_t) (p - slot); }
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        // (exec-masked for held lanes only: slower, profiles/r02_e)
        p[0] = (uint8_t) val;
        p[1] = (uint8_t) (val >> 16);
        p += nb;
    }
};

struct CountEmit
{
    uint32_t n;
    __device__ __forceinline__ void operator()(uint32_t, uint32_t nb)
    {
        n += nb;
    }
};

struct GlobalEmit                            // slow path: byte stores
{
    uint8_t *dst;
    uint32_t n;
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        if (nb >= 1)
            dst[n] = (uint8_t) val;
        if (nb == 2)
            dst[n + 1] = (uint8_t) (val >> 16);
        n += nb;
    }
};

// byte stores of the low nb (<= 3) bytes of v at d
__device__ __forceinline__ void
write_bytes(QH_LDS uint8_t *d, uint32_t v, uint32_t nb)
{
    if (nb > 0)
        d[0] = (uint8_t) v;
    if (nb > 1)
        d[1] = (uint8_t) (v >> 8);
    if (nb > 2)
        d[2] = (uint8_t) (v >> 16);
}

// ---- long strings: wave-cooperative decode ----
//
// One lane walks one string: a tile's time is its longest string's.  On the
// reference's own header corpora (tests/golden/data/*.qif) a tile's longest
// string is ~13x its mean one (cookies, user agents, 1,461-byte values), so
// the lanes idle.  The strings of more than kCoopMin Huffman bytes are
// decoded by the whole wave instead, all of a tile's at once: their bits cut
// into segments of S bits (a multiple of 32, >= kSegMin, at most 64
// segments in all), one per lane:
//   A  every lane walks its segment from the segment's first bit -- a guess:
//      only lane 0 starts on a code boundary -- and marks the bit of each
//      symbol start it passes in a bitmap (one bit per input bit);
//   B  lane j then walks on from its exit -- the first symbol start past its
//      segment -- into segment j + 1 until it reaches a marked bit: from
//      there on its walk and lane j + 1's are the same walk (decoding is a
//      function of the position), so lane j + 1's exit is exact if lane j's
//      was.  Lane 0's is; a lane whose predecessor's walk crossed its whole
//      segment without meeting its marks takes that walk's exit instead and
//      walks on again (rare; at most one round per segment).  Huffman codes
//      resynchronise after a median of ~31 bits on that corpus
//      (90th percentile ~160), so B costs a fraction of A;
//   then the symbols of segment j are the ones B counted before the meeting
//   point plus lane j's marks after it; a wave scan gives each segment's
//   output offset, and
//   W  every lane decodes its segment again from its now exact first symbol
//      start, into the string's arena slot at that offset, with the D3 checks.
// A string whose W finds an error (EOS code, bad padding), or whose counts
// or exits disagree, is decoded again by its own lane (decode_string_lds),
// so the result is always the one-lane result.  Cost: ~3 walks of S bits
// per string against one walk of the whole string.
#ifndef QH_COOP_MIN
#define QH_COOP_MIN 128
#endif
#ifndef QH_DEC_COOP                          // 0: every string by its lane
                                             // (full kernel too)
#define QH_DEC_COOP 1
#endif
constexpr uint32_t kCoopMin = QH_COOP_MIN;      // Huffman bytes
#ifndef QH_SEG_MIN
#define QH_SEG_MIN 64
#endif
// (round 5: 64, was 128 -- a tile whose long strings total under ~8k bits
// spreads them over twice the lanes; corpus decode 0.95x in 8 same-box
// pairs, 32 and the thresholds 96 / 160 / 192 no better,
// profiles/r05_coopsweep)
constexpr uint32_t kSegMin = QH_SEG_MIN;        // bits per segment
static_assert(kSegMin % 32 == 0 && kSegMin >= 64, "segment bits");
constexpr uint32_t kCoopDummy = 128;            // sink bytes, 2 per lane

enum WalkMode { kWalkMark, kWalkCheck, kWalkEmit };


// Walk the symbols of the staged stream src that start at [pos, lim) of the
// string ending at bitend (lim <= bitend; a walk that reaches the string's
// last < kWinBits bits decodes them padded, as decode_string_lds), one or
// two symbols a step; pos ends on the first symbol start >= lim (or where
// the walk stopped).  n counts the symbols.  Mark: set each symbol start's
// bit in bm (bit x - b0).  Check: stop on a symbol start whose bit is set
// (hit = 1).  Emit: store the symbols at dst, below dend (the bytes a step
// does not emit, or past dend, go to the lane's sink byte), hit = 1 on an
// error (D3).  A code the string
// cannot hold (EOS, or running past bitend) ends the walk there.
template <int Mode>
__device__ __forceinline__ void
seg_walk(const QH_LDS uint32_t *src, uint32_t &pos, uint32_t lim,
         uint32_t bitend, const QH_LDS uint32_t *s_win,
         const QH_LDS uint16_t *s_sorted, QH_LDS uint32_t *bm, uint32_t b0,
         QH_LDS uint8_t *dst, QH_LDS uint8_t *dend, QH_LDS uint8_t *sink,
         uint32_t &n, uint32_t &hit)
{
    uint32_t A, B, t, p, nx;
    {
        const uint32_t i0 = pos >> 5, sk = pos & 31;
        A = src[i0];
        const uint32_t a1 = src[i0 + 1];
        B = sk ? a1 : A;
        t = (32 - sk) & 31;
        p = sk ? i0 + 2 : i0 + 1;
        nx = src[p];
    }
    auto advance = [&](uint32_t c) {
        uint32_t tn;
        const bool cross = __builtin_sub_overflow(t, c, &tn);
        A = cross ? B : A;
        B = cross ? nx : B;
        t = tn & 31;
        p += cross ? 1u : 0u;
        nx = src[p];
    };
    auto marked = [&](uint32_t x, bool live) -> bool {
        const uint32_t r = x - b0;
        const uint32_t w = bm[live ? r >> 5 : 0u];
        return live & (((w >> (r & 31)) & 1u) != 0);
    };
    // (Mark) the bitmap word being filled, in a register: a lane's marks
    // lie in its own segment, whose words it owns whole (segments are
    // multiples of 32 bits from b0), and come in increasing order, so each
    // word is stored whole with plain stores -- no atomics, no lane branch
    uint32_t mi = (pos - b0) >> 5, mw = 0;
    auto mark = [&](uint32_t r, bool on) {
        const uint32_t wi = r >> 5;
        const bool nw = on & (wi != mi);
        mw = nw ? 0u : mw;
        mi = nw ? wi : mi;
        mw |= on ? 1u << (r & 31) : 0u;
    };
    auto hook = [&](uint32_t e, uint32_t nb, uint32_t l0) {
        if constexpr (Mode == kWalkMark)
        {
            const uint32_t r0 = pos - b0;
            mark(r0, nb >= 1);
            // the first symbol's word is complete if the second moves on
            const uint32_t r1 = r0 + l0;
            const bool two = nb == 2;
            if (two & ((r1 >> 5) != mi))
                bm[mi] = mw;
            mark(r1, two);
            if (nb >= 1)
                bm[mi] = mw;
        }
        else if constexpr (Mode == kWalkEmit)
        {
            QH_LDS uint8_t *a0 = ((nb >= 1) & (dst < dend)) ? dst : sink;
            QH_LDS uint8_t *a1 = ((nb == 2) & (dst + 1 < dend)) ? dst + 1 : sink;
            *a0 = (uint8_t) e;
            *a1 = (uint8_t) (e >> 16);
            dst += nb;
        }
        n += nb;
    };
    constexpr uint32_t kMain = kWinBits;
    uint32_t W = __builtin_amdgcn_alignbit(A, B, t);
    for (;;)
    {
        bool live;
        uint32_t e;
        do
        {
            live = (pos < lim) & (bitend - pos >= kMain);
            const uint32_t idx =
                ((W >> (32 - kWinBits - 2)) & (live ? 4u * (kWinSize - 1) : 0u))
                | (live ? 0u : 4u * kHoldIdx);
            e = *(const QH_LDS uint32_t *) ((const QH_LDS uint8_t *) s_win + idx);
            if constexpr (Mode == kWalkCheck)
            {
                const bool m = marked(pos, live);
                hit |= m ? 1u : 0u;
                lim = m ? pos : lim;
                e = m ? kHoldEntry : e;
            }
            const uint32_t ns = ent_ns(e), l0 = ent_l0(e);
            const bool cut = (ns == 2) & (pos + l0 >= lim);
            const uint32_t nb = cut ? 1u : ns;
            const uint32_t c = cut ? l0 : ent_c(e);
            hook(e, nb, l0);
            pos += c;
            advance(c);
            W = __builtin_amdgcn_alignbit(A, B, t);
        } while (__builtin_amdgcn_ballot_w64(live & (e >= (1u << 24))));
        // lanes stalled on a code of 14..30 bits
        const bool lng = (pos < lim) & (bitend - pos >= kMain);
        if (__builtin_expect(!__builtin_amdgcn_ballot_w64(lng), 1))
            break;
        uint32_t L;
        const uint32_t sym = long_code(W, s_sorted, &L);
        const bool rej = lng & ((sym == 256) | (L > bitend - pos));
        const bool ok = lng & !rej;
        if constexpr (Mode == kWalkEmit)
            hit |= rej ? 1u : 0u;
        lim = rej ? pos : lim;
        hook(sym, ok ? 1u : 0u, 0u);
        const uint32_t c = ok ? L : 0u;
        pos += c;
        advance(c);
        W = __builtin_amdgcn_alignbit(A, B, t);
    }
    // the string's last < kWinBits bits: at most two symbols, then padding
    {
        const uint32_t rem = bitend - pos;
        bool live = (pos < lim) & (rem < kMain);
        if constexpr (Mode == kWalkCheck)
        {
            const bool m = marked(pos, live);
            hit |= m ? 1u : 0u;
            live = live & !m;
        }
        const uint32_t w = W | (0xffffffffu >> (rem & 31));
        const uint32_t e = s_win[w >> (32 - kWinBits)];
        const uint32_t ns = ent_ns(e), ct = ent_c(e), l0 = ent_l0(e);
        const bool two = (ns == 2) & (ct <= rem);
        const bool one = !two & (ns != 0) & (l0 <= rem);
        const uint32_t c = live ? (two ? ct : (one ? l0 : 0u)) : 0u;
        hook(e, live ? (two ? 2u : (one ? 1u : 0u)) : 0u, l0);
        if constexpr (Mode == kWalkEmit)
        {
            const uint32_t r2 = rem - c;             // padding bits
            const uint32_t inv = ~(w << (c & 31));
            const bool pad_ok = r2 < 8
                             && (r2 == 0 || (inv >> ((32 - r2) & 31)) == 0);
            hit |= (live & !pad_ok) ? 1u : 0u;
        }
        pos += c;
    }
}

// popcount of the bits [r0, r1) of bm, every lane its own range (r1 <= r0
// for an empty one); no lane branches past the trip count
__device__ __forceinline__ uint32_t
bm_count(const QH_LDS uint32_t *bm, uint32_t r0, uint32_t r1)
{
    const uint32_t w0 = r0 >> 5;
    const uint32_t w1 = r1 > r0 ? (r1 + 31) >> 5 : w0;
    const uint32_t K = wave_max_dpp(w1 - w0);
    uint32_t c = 0;
    for (uint32_t k = 0; k < K; ++k)
    {
        const uint32_t w = w0 + k;
        uint32_t v = w < w1 ? bm[w] : 0u;
        v = k == 0 ? v >> (r0 & 31) : v;
        c += __builtin_popcount(v);
    }
    return c;
}

// Decode the strings of the tile flagged in `coop` (lane j: its string at
// bytes [rs, re) of the stage, its arena slot at arena + slot) with the whole
// wave at once: string j gets max(1, bits_j / S) segments of S bits (lanes
// in string order; S a multiple of 32, >= kSegMin, small enough that the
// segments fit 64 lanes), its bitmap (bits_j / 32 + 2 words, zeroed here)
// in its own arena slot, which W overwrites only after the counts: a slot
// holds 8/5 of the string's bytes, the bitmap 1/4 + 8 -- so any number of
// long strings fit, however full the arena (round 4 first put the bitmaps
// above the slots, where two 1,105-byte strings of a full tile did not
// fit and fell back to one lane each: 200k-cycle tiles on the QIF corpus)
// -- A, B, the counts and W as above, each lane on its own string.  sink:
// kCoopDummy bytes.  Returns, in lane j, string j's output
// length, or -1 when its own lane must decode it (an invalid string, or any
// disagreement); 0 elsewhere.
__device__ __forceinline__ int
coop_decode(const QH_LDS uint32_t *src, uint64_t coop, uint32_t rs,
            uint32_t re, uint32_t slot, QH_LDS uint8_t *arena,
            QH_LDS uint8_t *sink,
            const QH_LDS uint32_t *s_win, const QH_LDS uint16_t *s_sorted,
            const Coord *pc = nullptr)
{
    // (profiling) the wave's last cooperative call: iteration 15, slots 4-9
    auto stamp = [&](int k) {
#ifdef QHUFF_PROFILE
        if (pc)
            prof_stamp(*pc, kProfIters - 1, k);
#else
        (void) k;
        (void) pc;
#endif
    };
    stamp(4);
    const uint32_t lane = lane_id();
    const bool mine = (coop >> lane) & 1;
    const uint32_t nb = mine ? 8 * (re - rs) : 0u;
    const uint32_t ncoop = (uint32_t) __builtin_popcountll(coop);   // < 64
    // sum_j max(1, nb_j / S) <= tot / S + ncoop <= 64
    const uint32_t tot = read_lane(all_lanes(wave_incl_scan(nb)), 63);
    const uint32_t dv = 64 - ncoop;
    uint32_t S = ((((tot + dv - 1) / dv) + 31) & ~31u);
    S = S > kSegMin ? S : kSegMin;
    const uint32_t ns = mine ? (nb / S > 0 ? nb / S : 1u) : 0u;
    const uint32_t g = all_lanes(wave_incl_scan(ns)) - ns;   // first segment
    // this lane's string j and segment q
    uint32_t j = lane, gj = 0, nsj = 0;
    for (uint64_t m = coop; m; m &= m - 1)
    {
        const uint32_t c = (uint32_t) __builtin_ctzll(m);
        const uint32_t gc = read_lane(g, c), nc = read_lane(ns, c);
        const bool in = lane - gc < nc;
        j = in ? c : j;
        gj = in ? gc : gj;
        nsj = in ? nc : nsj;
    }
    const bool act = nsj != 0;
    const uint32_t q = lane - gj;
    const uint32_t rsj = all_lanes((uint32_t) __shfl((int) rs, (int) j, 64));
    const uint32_t rej = all_lanes((uint32_t) __shfl((int) re, (int) j, 64));
    const uint32_t slj = all_lanes((uint32_t) __shfl((int) slot, (int) j, 64));
    const uint32_t b0 = act ? 8 * rsj : 0u;
    const uint32_t b1 = act ? 8 * rej : 0u;
    QH_LDS uint8_t *sl = arena + slj;
    QH_LDS uint32_t *bm = (QH_LDS uint32_t *) (arena + ((slj + 3) & ~3u));
    const uint32_t s = act ? b0 + q * S : 0u;
    const uint32_t stop = !act ? 0u : q + 1 < nsj ? s + S : b1;
    {
        // each segment's lane zeroes its own words (S is a multiple of 32),
        // the last one the string's two spare words too
        const uint32_t wb = act ? (s - b0) >> 5 : 0u;
        const uint32_t we = !act ? 0u
                          : q + 1 < nsj ? (stop - b0) >> 5 : (b1 - b0) / 32 + 2;
        const uint32_t K = wave_max_dpp(we - wb);
        for (uint32_t k = 0; k < K; ++k)
            if (wb + k < we)
                bm[wb + k] = 0;
    }
    wave_sync();
    // A: guessed walks, marking
    uint32_t E = s, C = 0, h = 0;
    seg_walk<kWalkMark>(src, E, stop, b1, s_win, s_sorted, bm, b0, nullptr,
                        nullptr, sink, C, h);
    wave_sync();
    stamp(5);
    // B: walk on into the next segment of the string until meeting its marks
    const bool cl = act & (q + 1 < nsj);
    const uint32_t lim2 = !cl ? b1 : q + 2 < nsj ? s + 2 * S : b1;
    uint32_t cs = E, X = 0, K = 0, met = 0;
    bool redo = cl;
    uint32_t pm = 0, px = 0, rounds = 0;
    while (__builtin_amdgcn_ballot_w64(redo))
    {
        uint32_t x = redo ? cs : b1, k = 0, hm = 0;
        seg_walk<kWalkCheck>(src, x, redo ? lim2 : b1, b1, s_win, s_sorted, bm,
                             b0, nullptr, nullptr, sink, k, hm);
        X = redo ? x : X;
        K = redo ? k : K;
        met = redo ? hm : met;
        // segment q >= 1: its exact exit is its own (segment q - 1's walk met
        // its marks) or segment q - 1's walk's end
        pm = all_lanes(wave_shr1(met));
        px = all_lanes(wave_shr1(X));
        const uint32_t tE = (q >= 1 && !pm) ? px : E;
        redo = cl & (tE != cs);
        cs = cl ? tE : cs;
        if (++rounds > 64)                   // (cannot happen: segment q's
            return mine ? -1 : 0;            // exit is fixed after q rounds)
    }
    stamp(6);
#ifdef QHUFF_PROFILE
    if (pc)
        prof_value(*pc, kProfIters - 1, 9, rounds);
#endif
    // symbols of each segment, offsets within the string
    const uint32_t kp = all_lanes(wave_shr1(K));
    const bool cnt_own = act && q >= 1 && pm;
    const uint32_t own = bm_count(bm, cnt_own ? px - b0 : 0u,
                                  cnt_own ? stop - b0 : 0u);
    const uint32_t T = !act ? 0u : q == 0 ? C : kp + own;
    const uint32_t incl = all_lanes(wave_incl_scan(T));
    const uint32_t base = all_lanes((uint32_t) __shfl((int) (incl - T), (int) gj,
                                                      64));
    const uint32_t N = all_lanes((uint32_t) __shfl((int) incl,
                                                   (int) (gj + nsj - 1), 64))
                     - base;
    const bool big = N > (8 * ((b1 - b0) >> 3)) / 5;   // more than the slot
    stamp(7);
    // W: decode from the exact first symbol starts
    const uint32_t pcs = all_lanes(wave_shr1(cs));
    const uint32_t ts = q == 0 ? b0 : pcs;
    const bool wr = act & !big;
    uint32_t x = wr ? ts : b1, m = 0, bad = 0;
    seg_walk<kWalkEmit>(src, x, wr ? stop : b1, b1, s_win, s_sorted, bm, b0,
                        sl + (incl - T - base), sl + N, sink + 2 * lane, m,
                        bad);
    stamp(8);
    // each exit must be the next segment's start
    const uint32_t nts = all_lanes((uint32_t) __shfl_down((int) ts, 1, 64));
    const bool chain = q + 1 < nsj ? x == nts : true;
    const uint64_t fb = __builtin_amdgcn_ballot_w64(
        act & (big | (m != T) | (bad != 0) | !chain));
    // lane j: its string's segments gj .. gj + nsj - 1 (its own g, ns)
    const uint64_t segm = ns >= 64 ? ~0ull : ((1ull << ns) - 1) << g;
#ifdef QH_COOP_DEBUG
    // (diagnostic builds) a failing string's first failing segment, as 8
    // u32 at its slot: reason bits, q, m, T, exit, next start, S, segments
    for (uint64_t mm = coop; mm; mm &= mm - 1)
    {
        const uint32_t c = (uint32_t) __builtin_ctzll(mm);
        const uint32_t gc = read_lane(g, c), nc = read_lane(ns, c);
        const uint64_t sm_ = nc >= 64 ? ~0ull : ((1ull << nc) - 1) << gc;
        if (fb & sm_)
        {
            const uint32_t f0 = (uint32_t) __builtin_ctzll(fb & sm_);
            const uint32_t why = (read_lane(big ? 1u : 0u, f0))
                               | (read_lane(m != T ? 2u : 0u, f0))
                               | (read_lane(bad ? 4u : 0u, f0))
                               | (read_lane(chain ? 0u : 8u, f0));
            const uint32_t rec[8] = {why, read_lane(q, f0), read_lane(m, f0),
                                     read_lane(T, f0), read_lane(x, f0),
                                     read_lane(nts, f0), S, nc};
            QH_LDS uint8_t *d = arena + read_lane(slot, c);
            if (lane < 32)
                d[lane] = (uint8_t) (rec[lane >> 2] >> (8 * (lane & 3)));
        }
    }
#endif
    const uint32_t Nj = all_lanes((uint32_t) __shfl((int) N, (int) g, 64));
    return !mine ? 0 : (fb & segm) ? -1 : (int) Nj;
}

// copy n bytes src -> dst (LDS) with the whole wave: whole dwords at dst,
// the unaligned head and tail bytewise
__device__ __forceinline__ void
copy_wave(const QH_LDS uint8_t *src, QH_LDS uint8_t *dst, uint32_t n)
{
    const uint32_t lane = lane_id();
    uint32_t h = (4 - ((uint32_t) (uintptr_t) dst & 3)) & 3;
    h = h < n ? h : n;
    const uint32_t nb = (n - h) >> 2;
    const uint32_t it = h + 4 * nb;
    const uint32_t sb = (uint32_t) (uintptr_t) (src + h), r = sb & 3;
    const QH_LDS uint32_t *sw = (const QH_LDS uint32_t *) (src + h - r);
    QH_LDS uint32_t *dw = (QH_LDS uint32_t *) (dst + h);
    for (uint32_t i = lane; i < nb; i += 64)
        dw[i] = align_bytes(sw[i + 1], sw[i], r);
    if (lane < h)
        dst[lane] = src[lane];
    if (lane >= 4 && lane - 4 < n - it)
        dst[it + lane - 4] = src[it + lane - 4];
}

// Arena slot -> stage at byte D, for every lane of the wave at once, with
// whole dwords and no per-dword lane branches (the per-lane copy it replaced,
// with one lane branch per dword, is neutral-to-slower: profiles/r03_robust): each lane's body dwords go out in trips of
// eight, the trips and the dwords within them in DESCENDING order, and past
// its last body dword a lane stores garbage instead of branching.  Lane l's
// garbage lands only on dwords of later strings (its body starts at D_l <
// D_m for every later lane m with a body), and lane m stores its own dword
// X at index X - D_m < X - D_l, i.e. later in the descending order; the
// dwords shared by two strings (heads and tails) are written byte by byte
// after every body store.  (Each dword is its own store instruction: see
// below.)  Garbage past the tile's last string stays below
// the stage's end (fast tiles leave >= 64 bytes free).  One lane branch per
// trip instead of one per dword.
__device__ __forceinline__ void
compact_wave(const QH_LDS uint8_t *src, QH_LDS uint8_t *dstb, uint32_t n)
{
    uint32_t h = (4 - ((uint32_t) (uintptr_t) dstb & 3)) & 3;
    h = h < n ? h : n;
    const uint32_t nb = (n - h) >> 2;
    const uint32_t nt = n - h - 4 * nb;
    const uint32_t sa = (uint32_t) (uintptr_t) src;
    const QH_LDS uint32_t *sw = (const QH_LDS uint32_t *) (src - (sa & 3));
    const uint32_t s3 = sa & 3;
    const uint32_t it = h + 4 * nb;
    const uint32_t qt = (s3 + it) >> 2;
    const uint32_t vh = align_bytes(sw[1], sw[0], s3);
    const uint32_t vt = align_bytes(sw[qt + 1], sw[qt], (s3 + it) & 3);
    const uint32_t sb = s3 + h, r = sb & 3;
    const QH_LDS uint32_t *bw = sw + (sb >> 2);
    QH_LDS uint32_t *dw = (QH_LDS uint32_t *) (dstb + h);
    const uint32_t trips = (nb + 7) >> 3;
    const uint32_t K = wave_max_dpp(trips);
    for (uint32_t k = K; k-- > 0;)
    {
        if (k < trips)
        {
            uint32_t w[9];
#pragma unroll
            for (int j = 0; j < 9; ++j)
                w[j] = bw[8 * k + j];
            // one store instruction per dword, in this order: two dwords in
            // one ds_write2 would let a lane's garbage and another lane's
            // dword meet in one instruction (the compiler pairs neighbouring
            // stores and may reorder them; an empty asm with a memory
            // clobber between them stops both)
#pragma unroll
            for (int j = 7; j >= 0; --j)
            {
                dw[8 * k + j] = align_bytes(w[j + 1], w[j], r);
                asm volatile("" ::: "memory");
            }
        }
    }
    wave_sync();
    write_bytes(dstb, vh, h);
    write_bytes(dstb + it, vt, nt);
}



// A tile whose input or output does not fit the stage, coded eagerly:
// input staged -> the arena already holds the bytes (sz / st given);
// otherwise count from global memory, then decode again to global.  The
// tile's output base comes from base_of(total) (the batch kernel's look-back,
// or the service's running offset); its offsets and statuses go to t_off /
// t_status (the tile's first string).  Returns base + total.  Out of line
// (cold), state by value.  Keep: a rejected string's output is the bytes
// decoded before its error (DecPolicyT).
template <bool Keep, class SM, class BaseOf>
__device__ __noinline__ uint64_t
dec_slow_tile(const uint8_t *in, QH_LDS SM *sm, QH_LDS DecWave *wv,
              uint32_t slot0, uint32_t cnt, TileOffs to, Span sp, uint32_t sz,
              uint32_t st, bool sized, uint8_t *out, uint32_t *t_off,
              uint8_t *t_status, BaseOf base_of)
{
    const uint32_t lane = lane_id();
    const bool valid = lane < cnt;
    const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa) : 0;
    const uint32_t re = valid ? (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa) : 0;
    const DecGlb src{(const QH_GLB uint32_t *) sp.pa};
    if (!sp.staged && !sized)
    {
        int r = 0;
        if (valid)
        {
            CountEmit em{0};
            r = decode_string(src, 8 * rs, 8 * re, sm->win, sm->sorted, em);
        }
        sz = r >= 0 ? (uint32_t) r : Keep ? (uint32_t) (-1 - r) : 0u;
        st = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
    }
    const uint32_t incl = wave_incl_scan(sz);
    const uint32_t excl = incl - sz;
    const uint32_t total = read_lane(incl, 63);
    const uint64_t base = base_of(total);
    uint8_t *dst = out + base + excl;
    if (sp.staged)
    {
        const QH_LDS uint8_t *sa = wv->arena + slot0;
        for (uint32_t i = 0; i < sz; ++i)
            ((QH_GLB uint8_t *) dst)[i] = sa[i];
    }
    else if (valid && (Keep || st == QHUFF_DEC_OK) && sz)
    {
        GlobalEmit em{dst, 0};
        decode_string(src, 8 * rs, 8 * re, sm->win, sm->sorted, em);
    }
    if (valid)
    {
        ((QH_GLB uint32_t *) t_off)[lane] = (uint32_t) (base + excl);
        ((QH_GLB uint8_t *) t_status)[lane] = (uint8_t) st;
    }
    return base + total;
}


// The sizes (and statuses) of a tile past the stage, counted in global
// memory, as dec_slow_tile counts them (sized = false)
struct SzSt
{
    uint32_t sz, st;
};
template <bool Keep, class SM>
__device__ __noinline__ SzSt
dec_tile_sizes(const uint8_t *in, QH_LDS SM *sm, uint32_t cnt, TileOffs to,
               Span sp)
{
    const bool valid = lane_id() < cnt;
    int r = 0;
    if (valid)
    {
        const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa);
        const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa);
        const DecGlb src{(const QH_GLB uint32_t *) sp.pa};
        CountEmit em{0};
        r = decode_string(src, 8 * rs, 8 * re, sm->win, sm->sorted, em);
    }
    SzSt o;
    o.sz = r >= 0 ? (uint32_t) r : Keep ? (uint32_t) (-1 - r) : 0u;
    o.st = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
    return o;
}

template <bool Keep, class SM>
__device__ __forceinline__ bool
dec_big_sizes(const uint8_t *in, QH_LDS SM *sm, QH_LDS DecWave *wv,
              uint32_t cnt, TileOffs to, Span sp, uint32_t &sz, uint32_t &st,
              uint32_t slot0, uint8_t *dst);

// the decode side of the wave pipeline (qhuff_pipeline.h, qhuff_service.hip);
// SM: the workgroup's LDS (win, sorted).  Keep (the kernel the per-string
// entry points use to replay where the reference stops on an invalid
// string, qhuff_shim.cpp): a rejected string keeps, as its output, the bytes
// decoded before the error; its status is QHUFF_DEC_ERROR all the same.
template <class SM, bool Keep = false, bool Full = true>
struct DecPolicyT
{
    static constexpr bool kStatus = true;
    // Full: the kernel for batches with big tiles (output slots) and long
    // strings (coop_phase after the codec); the lean one codes those tiles
    // out of line and its strings by their lanes, and its hot loop keeps its
    // registers (qhuff_host.cpp picks the kernel per launch)
    static constexpr bool kBig = Full;
    static constexpr bool kCoop = Full && QH_DEC_COOP;
    static constexpr int kInCap = kDecInCap;
    static constexpr int kDepth = QH_DEPTH;       // pending tiles
    static constexpr int kOutCap = kDecStageCap;
    static constexpr int kNch = kDecNch;          // 16-byte chunks per lane
    static constexpr uint32_t kTS = kDecTS;       // strings per tile
    using Offs = TileOffs;
    const uint8_t *in;
    QH_LDS SM *sm;
    QH_LDS DecWave *wv;
    uint32_t slot0;                  // this lane's arena slot (current tile)
    uint64_t coop = 0;               // strings decoded by the whole wave
#ifdef QHUFF_PROFILE
    const Coord *pc = nullptr;       // (profiling) stamps of coop_decode
#endif

    __device__ __forceinline__ void stage_in(const Chunks<kNch> &ch,
                                             const Span &sp, const Offs &)
    {
        ch.store<true>((QH_LDS u32x4 *) wv->in, sp.n16);
    }
    __device__ __forceinline__ void prepare(const Span &) {}
    __device__ __forceinline__ const QH_LDS uint32_t *out_stage() const
    {
        return wv->in;
    }
    // staged tile: decode this lane's string into its arena slot; strings
    // above kCoopMin Huffman bytes with the whole wave (coop_decode), when
    // their bitmap fits in the arena past the slots
    __device__ __forceinline__ void codec(const Offs &to, uint32_t cnt,
                                          const Span &sp, uint32_t *sz,
                                          uint32_t *st)
    {
        codec_range(to, 0, cnt, sp, sz, st);
    }
    // the strings of lanes [lo, hi) (sp: their span)
    __device__ __forceinline__ void codec_range(const Offs &to, uint32_t lo,
                                                uint32_t cnt, const Span &sp,
                                                uint32_t *sz, uint32_t *st)
    {
        const uint32_t lane = lane_id();
        const bool valid = (lane >= lo) & (lane < cnt);
        const uint32_t A = read_lane(to.o0, lo);
        const uint32_t hl = to.o1 - to.o0;
        const bool fixed = !__builtin_amdgcn_ballot_w64(
            valid & (hl > kFixMaxLen));
        slot0 = fixed ? kFixStride * lane
                      : 2 * lane + (uint32_t) ((8ull * (to.o0 - A)) / 5);
        const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa);
        const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa);
        // the slots end below kVarArenaBytes - slack + 1 for this span; the
        // bitmap (hl / 4 + 2 words) and the sinks go above them
        // (at most 48 cooperative strings: at least 16 lanes for segments)
        const bool cand = kCoop && !fixed && valid && hl > kCoopMin;
        coop = __builtin_amdgcn_ballot_w64(cand);
        if (__builtin_popcountll(coop) > 48)
            coop = 0;
        const bool mine = (coop >> lane) & 1;
        int r = 0;
        if (valid)
        {
            ArenaEmit em{wv->arena + slot0, wv->arena + slot0, 0};
            r = decode_string_lds(wv->in, 8 * rs, mine ? 8 * rs : 8 * re,
                                  sm->win, sm->sorted, sm->long2, em);
        }
        *sz = r >= 0 ? (uint32_t) r : Keep ? (uint32_t) (-1 - r) : 0u;
        *st = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
    }
    // The strings flagged in `coop` by the codec, with the whole wave
    // (coop_decode), into their sizes and statuses.  A separate step: the
    // tile loop first moves its pending tiles' outputs out of registers
    // (qhuff_pipeline.h), so this code runs beside few live values.
    __device__ __forceinline__ void coop_phase(const Offs &to, uint32_t lo,
                                               uint32_t cnt, const Span &sp,
                                               uint32_t *sz, uint32_t *st)
    {
        const uint32_t lane = lane_id();
        const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa);
        const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa);
        const bool mine = (coop >> lane) & 1;
#ifdef QH_COOP_DEBUG
        bool dbg_fb = false;
#endif
        int r = 0;
        const int rc = coop_decode(
            wv->in, coop, rs, re, slot0, wv->arena,
            wv->arena + kArenaBytes - kCoopDummy, sm->win, sm->sorted
#ifdef QHUFF_PROFILE
            , pc
#endif
            );
        r = rc;
        const uint64_t fail = __builtin_amdgcn_ballot_w64(mine & (rc < 0));
#ifdef QH_COOP_DEBUG
        if (fail)
        {
            const bool f = (fail >> lane) & 1;
            r = f ? 32 : r;
            dbg_fb = f;
            coop &= ~fail;
        }
        if (false)
#else
        if (fail)
#endif
        {
            // (rare) an invalid string: its own lane decodes it again
            // (the other lanes' two stores go to their sink bytes)
            coop &= ~fail;
            const bool f = (fail >> lane) & 1;
            QH_LDS uint8_t *d0 = f ? wv->arena + slot0
                                   : wv->arena + kArenaBytes - kCoopDummy
                                         + 2 * lane;
            ArenaEmit em{d0, d0, 0};
            const int r2 = decode_string_lds(wv->in, 8 * rs,
                                             f ? 8 * re : 8 * rs, sm->win,
                                             sm->sorted, sm->long2, em);
            r = f ? r2 : r;
        }
        if (mine)
        {
            *sz = r >= 0 ? (uint32_t) r : Keep ? (uint32_t) (-1 - r) : 0u;
            *st = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
#ifdef QH_COOP_DEBUG
            *st = dbg_fb ? 7u : *st;
#endif
        }
    }
    // arena -> the (dead) input stage, compacted (the cooperative strings
    // by the whole wave, after the rest)
    __device__ __forceinline__ void emit(uint32_t excl, uint32_t sz, uint32_t)
    {
#ifdef QH_TIME_NO_EMIT                       // timing builds only: no output
        return;
#endif
        QH_LDS uint8_t *stage = (QH_LDS uint8_t *) wv->in;
        compact_wave(wv->arena + slot0, stage + excl,
                     (coop >> lane_id()) & 1 ? 0u : sz);
        if (coop)
        {
            wave_sync();
            uint64_t m = coop;
            while (m)
            {
                const uint32_t j = (uint32_t) __builtin_ctzll(m);
                m &= m - 1;
                copy_wave(wv->arena + read_lane(slot0, j),
                          stage + read_lane(excl, j), read_lane(sz, j));
            }
        }
    }

    // a tile of the batch kernel: base from the look-back
    // a big tile's sizes, and its output into dst when it fits
    __device__ __forceinline__ bool big_sizes(uint32_t cnt, Offs to, Span sp,
                                              uint32_t &sz, uint32_t &st,
                                              uint8_t *dst)
    {
#if QH_COOP_VIA_BIG
        // a staged tile whose codec left strings for the whole wave
        // (qhuff_pipeline.h): their cooperative phase here
        if (kCoop && sp.staged && coop)
            coop_phase(to, 0, cnt, sp, &sz, &st);
#endif
        return dec_big_sizes<Keep>(in, sm, wv, cnt, to, sp, sz, st, slot0, dst);
    }
    // a big tile whose output does not fit a slot (qhuff_pipeline.h), after
    // the pending tiles are flushed: base from the look-back
    // the sizes of a tile past the stage (the lean kernel: no codec ran)
    __device__ __forceinline__ void slow_size(uint32_t cnt, Offs to, Span sp,
                                              uint32_t &sz, uint32_t &st)
    {
        const SzSt r = dec_tile_sizes<Keep>(in, sm, cnt, to, sp);
        sz = r.sz;
        st = r.st;
    }
    // ... its output once the look-back lb (aggregate published) resolves
    __device__ __forceinline__ void slow_tile(Coord c, uint32_t t, uint32_t cnt,
                                              Offs to, Span sp, uint32_t sz,
                                              uint32_t st, bool sized,
                                              uint8_t *out, uint32_t *out_off,
                                              uint8_t *status, uint64_t n,
                                              const LookBack &lb)
    {
        const uint64_t s0 = (uint64_t) t * kTS;
        const uint64_t end = dec_slow_tile<Keep>(in, sm, wv, slot0, cnt, to,
                                                    sp, sz, st, sized, out,
                                                    out_off + s0, status + s0,
                                                    StartedBase{c, lb});
        last_tile_end(c, t, end, out_off, n);
    }
    // a tile at a known base
    __device__ __forceinline__ uint64_t slow_tile_at(uint64_t base, uint32_t cnt,
                                                     Offs to, Span sp, uint32_t sz,
                                                     uint32_t st, uint8_t *out,
                                                     uint32_t *t_off,
                                                     uint8_t *t_status)
    {
        return dec_slow_tile<Keep>(in, sm, wv, slot0, cnt, to, sp, sz, st,
                                      false, out, t_off, t_status,
                                      FixedBase{base});
    }
};


// The sizes of a big tile (statuses too) and, when they fit kBigSlotBytes,
// its whole compacted output at dst (a big-tile slot, qhuff_pipeline.h),
// written before its base is known: the tile then waits for its look-back
// like any other, and its wave goes on coding.  Staged input: the main
// codec has sized and decoded it into the arena (sz, st, slot0 given).
// Otherwise unit by unit, each staged, decoded into the arena and copied
// from there; a string whose input alone exceeds the stage is walked in
// global memory (into dst when its bound fits).  Returns whether all of
// the output went to dst; the sizes are complete either way.
template <bool Keep, class SM>
__device__ __forceinline__ bool
dec_big_sizes(const uint8_t *in, QH_LDS SM *sm, QH_LDS DecWave *wv,
              uint32_t cnt, TileOffs to, Span sp, uint32_t &sz, uint32_t &st,
              uint32_t slot0, uint8_t *dst)
{
    using P = DecPolicyT<SM, Keep, true>;
    P pol{in, sm, wv, 0};
    const uint32_t lane = lane_id();
    uint32_t run = 0;                        // output bytes so far (uniform)
    bool fits = true;
    // the arena slots of lanes [lo, hi) -> dst + run, compacted
    auto put = [&](uint32_t lo, uint32_t hi, uint32_t s, uint32_t t,
                   uint32_t slot) {
        const bool in_u = (lane >= lo) & (lane < hi);
        const uint32_t ls = (in_u && (Keep || t == QHUFF_DEC_OK)) ? s : 0u;
        const uint32_t incl = all_lanes(wave_incl_scan(ls));
        const uint32_t ut = read_lane(incl, 63);
        fits = fits && run + ut <= kBigSlotBytes;
        if (fits)
        {
            const bool lng = ls > 64;
            if (ls && !lng)
            {
                const QH_LDS uint8_t *sa = wv->arena + slot;
                uint8_t *d = dst + run + (incl - ls);
                for (uint32_t i = 0; i < ls; ++i)
                    ((QH_GLB uint8_t *) d)[i] = sa[i];
            }
            for (uint64_t m = __builtin_amdgcn_ballot_w64(lng); m; m &= m - 1)
            {
                const uint32_t j = (uint32_t) __builtin_ctzll(m);
                copy_out(wv->arena + read_lane(slot, j),
                         dst + run + read_lane(incl - ls, j), read_lane(ls, j));
            }
        }
        run += ut;
    };
    if (sp.staged)
    {
        put(0, cnt, sz, st, slot0);
        return fits;
    }
    sz = 0;
    st = 0;
    for (uint32_t i0 = 0; i0 < cnt;)
    {
        const uint32_t k = unit_len(in, to, i0, cnt, P::kInCap, false, 0, 0, 0);
        if (k == 0)
        {
            // one string beyond the stage: its lane walks it in global memory
            const uintptr_t pa = (uintptr_t) (in + read_lane(to.o0, i0))
                               & ~(uintptr_t) 15;
            const DecGlb src{(const QH_GLB uint32_t *) pa};
            const uint32_t rs = (uint32_t) ((uintptr_t) (in + to.o0) - pa);
            const uint32_t re = (uint32_t) ((uintptr_t) (in + to.o1) - pa);
            const uint32_t bound = (8 * read_lane(re - rs, i0)) / 5 + 1;
            const bool w = fits && run + bound <= kBigSlotBytes;
            int r = 0;
            if (lane == i0)
            {
                if (w)
                {
                    GlobalEmit em{dst + run, 0};
                    r = decode_string(src, 8 * rs, 8 * re, sm->win, sm->sorted,
                                      em);
                }
                else
                {
                    CountEmit em{0};
                    r = decode_string(src, 8 * rs, 8 * re, sm->win, sm->sorted,
                                      em);
                }
                sz = r >= 0 ? (uint32_t) r : Keep ? (uint32_t) (-1 - r) : 0u;
                st = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
            }
            fits = w;
            run += read_lane(sz, i0);
            i0 += 1;
            continue;
        }
        const Span su = tile_span(in, read_lane(to.o0, i0),
                                  read_lane(to.o1, i0 + k - 1), P::kInCap);
        stage_chunks<true>(su, (QH_LDS u32x4 *) wv->in);
        uint32_t s1, t1;
        pol.codec_range(to, i0, i0 + k, su, &s1, &t1);
        if (pol.coop)
            pol.coop_phase(to, i0, i0 + k, su, &s1, &t1);
        wave_sync();
        put(i0, i0 + k, s1, t1, pol.slot0);
        if ((lane >= i0) & (lane < i0 + k))
        {
            sz = s1;
            st = t1;
        }
        wave_sync();
        i0 += k;
    }
    return fits;
}

}  // namespace qhuff
