// qhuff_decode.hip -- batch Huffman decode kernel (gfx950).
//
// Reference path:
//   D1 lsqpack_huff_decode  lsqpack.c:3520-3535 (resume == 0 && final)
//   D2 huff_decode_fast     lsqpack.c:5234-5466 (16-bit window table, slow
//                           path to the nibble FSM for long codes)
//   D3 accept/reject rule: ERROR iff the EOS code occurs, or the bits after
//      the last complete symbol are >= 8 or not all ones
//      (lsqpack.c:5362-5426, 3482-3497)
//
// One string per lane, one 64-string tile per wave (qhuff_device.h).  The
// tile's input is staged in the wave's LDS region as big-endian dwords;
// each lane keeps a 64-bit bit buffer in registers, refilled from the stage
// one aligned dword at a time (the refill read is independent of the table
// lookup, so one LDS round trip sits on the per-step dependency chain).  A
// step looks the top 12 bits up in a window table (up to two symbols of
// <= 12 bits); codes of 13..30 bits take a canonical length search behind a
// wave-uniform branch.  While >= 32 real bits remain the step needs no
// padding or tail logic; the last < 32 bits run a careful epilogue that
// pads with ones (as huff_decode_fast pads its last window,
// lsqpack.c:5364-5365) and applies the D3 rule.
//
// Output bytes land in a byte-granular per-string arena slot.  After the
// wave scan of the sizes they are compacted into the (now dead) input stage
// and copied out with 16-byte stores once the look-back has resolved the
// tile's output base.
#include "qhuff_kernels.h"

namespace qhuff {

constexpr int kDecWaves = 16;                          // waves per workgroup
constexpr int kDecInCap = 3072;                        // staged input bytes
// byte slot of string i: 2i + floor(8 * (rs_i - A) / 5) -- an output is at
// most 8/5 of its input, plus one byte written past the end by the
// two-byte emitter
constexpr int kArenaBytes = 2 * kWT + 8 * kDecInCap / 5 + 32;
constexpr int kDecChunks = kDecInCap / 16 / 64;        // 16-B chunks per lane
constexpr int kDecOutChunks = 3;                       // covers a stage of 3072 B

struct DecWave                       // one wave's private LDS region
{
    alignas(16) uint32_t in[kDecInCap / 4];   // BE input dwords; output stage
    alignas(16) uint8_t arena[kArenaBytes];
};

struct DecSmem
{
    uint32_t win[kWinSize];
    uint16_t sorted[257];
    DecWave w[kDecWaves];
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
        const uint32_t el = (sym & 0xff) | (L << 16) | (1u << 24)
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
// output bytes, or -1 for a rejected string.  Three wave-uniform phases:
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
        const uint32_t ns = (e >> 24) & 3, ct = (e >> 16) & 15,
                       l0 = (e >> 20) & 15;
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
    return bad ? -1 : (int) emit.n;
}

// byte-granular arena sink: two unconditional byte stores per step (the
// second is overwritten by the next step when only one symbol was emitted)
struct ArenaEmit
{
    QH_LDS uint8_t *slot;
    uint32_t n;
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        slot[n] = (uint8_t) val;
        slot[n + 1] = (uint8_t) (val >> 8);
        n += nb;
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
            dst[n + 1] = (uint8_t) (val >> 8);
        n += nb;
    }
};

// per-lane string bounds of a tile relative to its span
struct LaneStr
{
    bool valid;
    uint32_t rs, re;                 // byte positions relative to span.pa
    uint32_t slot0;                  // arena slot
};

__device__ __forceinline__ LaneStr
lane_str(const uint8_t *in, const TileOffs &to, uint32_t cnt, const Span &sp)
{
    LaneStr ls;
    const uint32_t lane = lane_id();
    ls.valid = lane < cnt;
    const uint32_t A = to.first();
    ls.rs = ls.valid ? (uint32_t) ((uintptr_t) (in + to.o0) - sp.pa) : 0;
    ls.re = ls.valid ? (uint32_t) ((uintptr_t) (in + to.o1) - sp.pa) : 0;
    ls.slot0 = 2 * lane + (uint32_t) ((8ull * (to.o0 - A)) / 5);
    return ls;
}

// arena slot -> stage at byte D (wave-synchronous; other lanes write the
// neighbouring bytes): bytes up to a dword boundary, whole dwords, tail
__device__ __forceinline__ void
compact_string(const QH_LDS uint8_t *src, QH_LDS uint8_t *dstb, uint32_t n)
{
    uint32_t h = (4 - ((uint32_t) (uintptr_t) dstb & 3)) & 3;
    h = h < n ? h : n;
    for (uint32_t i = 0; i < h; ++i)
        dstb[i] = src[i];
    const QH_LDS uint8_t *s2 = src + h;
    const uint32_t s3 = (uint32_t) ((uintptr_t) s2 & 3);
    const QH_LDS uint32_t *sw = (const QH_LDS uint32_t *) (s2 - s3);
    QH_LDS uint32_t *dw = (QH_LDS uint32_t *) (dstb + h);
    const uint32_t nb = (n - h) >> 2;
    for (uint32_t k = 0; k < nb; ++k)
        dw[k] = align_bytes(sw[k + 1], sw[k], s3);
    for (uint32_t i = h + 4 * nb; i < n; ++i)
        dstb[i] = src[i];
}

__global__ __launch_bounds__(64 * kDecWaves) void
qhuff_decode_kernel(DecArgs a)
{
    __shared__ DecSmem smem;
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    const int tid = threadIdx.x;
    {
        const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) glb(a.win);
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
        for (int i = tid; i < kWinSize / 4; i += 64 * kDecWaves)
            sw[i] = gw[i];
        const QH_GLB uint16_t *gs = glb(a.sorted);
        if (tid < 257)
            sm->sorted[tid] = gs[tid];
        clear_next_launch(a.c);
    }
    __syncthreads();                 // the only workgroup barrier

    const uint32_t lane = lane_id();
    QH_LDS DecWave *wv = &sm->w[tid >> 6];
    QH_LDS uint32_t *stage = wv->in;
    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    QH_GLB uint32_t *gout_off = glb(a.out_off);
    QH_GLB uint8_t *gstat = glb(a.status);
    const uint32_t n_waves = gridDim.x * kDecWaves;
    const uint32_t gid = wave_gid(kDecWaves);
    const uint32_t nt = a.c.n_tiles;
    const uint32_t dbg = a.c.dbg;

    auto tile_cnt = [&](uint32_t t) -> uint32_t {
        return (uint32_t) min((uint64_t) kWT, a.n - (uint64_t) t * kWT);
    };

    // Tiles are claimed just in time: a wave claims its next tile only when
    // it is about to code it, so claim order is processing order and a
    // look-back only ever waits on tiles whose codec is already running.
    // The claim -> offsets -> input latency of one wave hides under the
    // codec work of the other waves on its SIMD.
    PhaseClock clk;
    clk.init(dbg);
    for (;;)
    {
        const uint32_t t = claim_tile(a.c, gid, n_waves);
        clk.lap(0);
        if (t >= nt)
            break;
        const uint32_t cnt = tile_cnt(t);
        TileOffs to;
        to.load(gin_off, (uint64_t) t * kWT, cnt);
        const Span sp = tile_span(a.in, to.first(), to.last(), kDecInCap);
        if (sp.staged)
        {
            Chunks<kDecChunks> ch;
            ch.load(sp);
            ch.store<true>((QH_LDS u32x4 *) stage, sp.n16);
        }
        wave_sync();
        clk.lap(1);

        // 1. decode this tile (input staged in LDS, or read from global)
        const LaneStr ls = lane_str(a.in, to, cnt, sp);
        int r = 0;
        if (ls.valid)
        {
            if (dbg & kDbgNoCodec)
                r = (int) (ls.re - ls.rs);
            else if (sp.staged)
            {
                ArenaEmit em{wv->arena + ls.slot0, 0};
                r = decode_string(DecLds{stage}, 8 * ls.rs, 8 * ls.re, sm->win,
                                  sm->sorted, em);
            }
            else
            {
                CountEmit em{0};
                r = decode_string(DecGlb{(const QH_GLB uint32_t *) sp.pa},
                                  8 * ls.rs, 8 * ls.re, sm->win, sm->sorted,
                                  em);
            }
        }
        const uint32_t sz = r < 0 ? 0u : (uint32_t) r;
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t excl = incl - sz;
        clk.lap(2);
        const uint32_t total = read_lane(incl, 63);

        // 2. publish the aggregate, issue the first look-back poll
        LookBack lb;
        if (!(dbg & kDbgNoLookback))
            lb.start(a.c, t, total);
        clk.lap(3);

        // 3. compaction: arena slots -> the (dead) input stage
        const bool staged_out = sp.staged && total + 64 <= (uint32_t) kDecInCap;
        wave_sync();
        if (staged_out && sz && !(dbg & kDbgNoCodec))
            compact_string(wv->arena + ls.slot0,
                           (QH_LDS uint8_t *) stage + 16 + excl, sz);
        wave_sync();

        clk.lap(4);

        // 4. output base
        const uint64_t base = (dbg & kDbgNoLookback) ? (uint64_t) t << 13
                            : lb.finish(a.c);
        clk.lap(5);

        // 5. copy-out (stage -> registers -> 16-byte stores)
        CopyOut<kDecOutChunks> co;
        if (staged_out)
            co.gather(stage, a.out + base, total);
        if (!(dbg & kDbgNoStore))
        {
            if (staged_out)
                co.store();
            else if (sz && sp.staged)
            {
                // output larger than the stage: arena -> global, bytes
                const QH_LDS uint8_t *src = wv->arena + ls.slot0;
                QH_GLB uint8_t *dst = (QH_GLB uint8_t *) (a.out + base + excl);
                for (uint32_t i = 0; i < sz; ++i)
                    dst[i] = src[i];
            }
            else if (sz && !(dbg & kDbgNoCodec))
            {
                // input larger than the stage: decode again, to global
                GlobalEmit em{a.out + base + excl, 0};
                decode_string(DecGlb{(const QH_GLB uint32_t *) sp.pa},
                              8 * ls.rs, 8 * ls.re, sm->win, sm->sorted,
                              em);
            }
            const uint64_t s0 = (uint64_t) t * kWT;
            if (ls.valid)
            {
                gout_off[s0 + lane] = (uint32_t) (base + excl);
                gstat[s0 + lane] = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
            }
            if (t == nt - 1 && lane == 0)
                gout_off[a.n] = (uint32_t) (base + total);
        }
        wave_sync();
        clk.lap(6);
    }
    clk.flush(a.c.err);
}

hipError_t
launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_decode_kernel, dim3(grid), dim3(64 * kDecWaves),
                       0, st, a);
    return hipGetLastError();
}

hipError_t
decode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_decode_kernel),
        64 * kDecWaves, 0);
}

int
decode_waves_per_block()
{
    return kDecWaves;
}

size_t
decode_lds_bytes()
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(qhuff_decode_kernel))
            != hipSuccess)
        return 0;
    return fa.sharedSizeBytes;
}

}  // namespace qhuff
