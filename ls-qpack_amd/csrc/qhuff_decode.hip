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
// One string per lane.  The tile's input is staged in LDS as big-endian
// dwords; each lane keeps a 64-bit bit buffer in registers, refilled from
// the stage one aligned dword at a time (the refill read is independent of
// the table lookup, so one LDS round trip sits on the per-step dependency
// chain).  A step looks the top 12 bits up in a window table (up to two
// symbols of <= 12 bits); codes of 13..30 bits take a canonical length
// search behind a wave-uniform branch.  While >= 32 real bits remain the
// step needs no padding or tail logic; the last < 32 bits run a careful
// epilogue that pads with ones (as huff_decode_fast pads its last window,
// lsqpack.c:5364-5365) and applies the D3 rule.
//
// Output bytes land in a byte-granular per-string arena slot.  After the
// workgroup scan the slots are compacted into an LDS output stage; the
// tile's look-back and copy-out are deferred to the workgroup's next
// iteration, when every predecessor has long published its aggregate
// (persistent grid, static tile assignment t = blockIdx.x + k * gridDim.x).
#include "qhuff_kernels.h"

namespace qhuff {

constexpr int kDecInCap = 7680;                        // staged input bytes
constexpr int kDecOutCap = 10 * 1024;                  // staged output bytes
// byte slot of string i: 2i + floor(8 * (rs_i - A) / 5) -- an output is at
// most 8/5 of its input, plus one byte written past the end by the
// two-byte emitter
constexpr int kArenaBytes = 2 * kTile + 8 * kDecInCap / 5 + 16;

struct DecSmem
{
    uint32_t win[kWinSize];
    uint16_t sorted[257];
    LongLen longc[kMaxLong];         // canonical long-code params
    uint32_t off[2][kTile + 1];      // current / next tile offsets
    uint32_t size[kTile];            // bit 31: rejected string
    uint32_t excl_p[kTile];          // tile offsets of the deferred tile
    uint32_t cnt[kBuckets];
    uint16_t perm[kTile];
    uint8_t stat_p[kTile];           // status of the deferred tile
    LdsScratch scr;
    alignas(16) uint32_t in[kDecInCap / 4 + 8];        // big-endian dwords
    alignas(16) uint32_t out[(kDecOutCap + 64) / 4];   // 16 B pad in front
    alignas(16) uint8_t arena[kArenaBytes];
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

// long-code step: canonical search over code lengths 13..30 (uniform table,
// unrolled selects)
__device__ __forceinline__ uint32_t
long_code(uint32_t w, const QH_LDS LongLen *lc, const QH_LDS uint16_t *s_sorted,
          uint32_t *len)
{
    uint32_t L = 0, idx = 0;
#pragma unroll
    for (int i = 0; i < kMaxLong; ++i)
    {
        // lengths past lp.n are padded with count 0 (never hit); uniform
        // LDS addresses (broadcast reads)
        const u32x4 ll = ((const QH_LDS u32x4 *) lc)[i];   // len first count base
        uint32_t v = w >> (32 - ll.x);
        uint32_t off = v - ll.y;
        bool hit = (L == 0) & (off < ll.z);
        L = hit ? ll.x : L;
        idx = hit ? ll.w + off : idx;
    }
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
          const QH_LDS uint16_t *s_sorted, const QH_LDS LongLen *lp, Emit &emit)
{
    uint32_t e = s_win[hi >> (32 - kWinBits)];
    bool ok = true;
    if (__builtin_amdgcn_ballot_w64((GATED ? act : true) & (e < (1u << 24))))
    {
        // a code of 13..30 bits: synthesize the entry of a one-symbol step
        uint32_t L;
        const uint32_t sym = long_code(hi, lp, s_sorted, &L);
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
              const QH_LDS LongLen *lp, Emit &emit)
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
                                         s_sorted, lp, emit);
        bad |= !ok;
        rem = ok ? rem : 0u;                 // leave phase 1 (rare)
    } while (!__builtin_amdgcn_ballot_w64(rem < 32));
    bool act = rem >= 32 && !bad;
    if (__builtin_amdgcn_ballot_w64(act))
    do
    {
        const uint32_t d = src.dw_ahead(p, bitend);
        const bool ok = main_step<true>(act, d, hi, lo, bits, rem, p, s_win,
                                        s_sorted, lp, emit);
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
            const uint32_t sym = long_code(w, lp, s_sorted, &L);
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

constexpr int kDecChunks = (kDecInCap / 16 + kLoadThreads - 1) / kLoadThreads;

// the unit whose look-back / copy-out is deferred to the next iteration
struct Deferred
{
    uint32_t tile, lo, hi;     // strings [lo, hi) of `tile`
    uint32_t total;            // output bytes of the unit
    uint32_t unit_off;         // output bytes of the tile's earlier units
    uint32_t staged_out;       // output sits in sm->out (else re-decode)
    bool first, last;          // first / last unit of its tile
};

// look-back wave: the deferred unit's output base.  The first unit of a
// tile resolves the tile's base by look-back; the last one publishes the
// tile's inclusive prefix (a one-unit tile does both in look_back_wave).
__device__ __forceinline__ uint64_t
resolve_unit_base(const Coord &c, const Deferred &df, int64_t *known_tile,
                  uint64_t *known_incl, uint64_t *tile_base)
{
    if (df.first)
    {
        uint32_t polls = 0;
        stamp(c, df.tile, 11);
        *tile_base = (c.dbg & kDbgNoLookback) ? (uint64_t) df.tile << 16
            : look_back_wave(c, df.tile, df.total, *known_tile, *known_incl,
                             &polls, df.last);
        stamp(c, df.tile, 12);
        stamp_value(c, df.tile, 14, polls);
    }
    const uint64_t ub = *tile_base + df.unit_off;
    if (df.last)
    {
        if (!df.first && !(c.dbg & kDbgNoLookback) && (threadIdx.x & 63) == 0)
            __hip_atomic_store(&c.flags[df.tile],
                               kFlagInc | ((uint64_t) c.epoch << 40)
                                        | ((ub + df.total) & kValMask),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *known_tile = df.tile;
        *known_incl = ub + df.total;
    }
    return ub;
}

// every thread: copy-out, offsets and status of the deferred unit; a unit
// whose output did not fit the LDS stage is decoded again by every lane
// straight to global memory (input read from global)
__device__ __forceinline__ void
finish_unit(const DecArgs &a, QH_LDS DecSmem *sm, const Deferred &df,
            uint64_t base)
{
    const int tid = threadIdx.x;
    if (a.c.dbg & kDbgNoStore)
        return;
    const uint32_t ucnt = df.hi - df.lo;
    const uint64_t s0 = (uint64_t) df.tile * kTile + df.lo;
    QH_GLB uint32_t *gout_off = glb(a.out_off);
    QH_GLB uint8_t *gstat = glb(a.status);
    if (df.staged_out)
        copy_out(sm->out, a.out + base, df.total);
    else if (tid < (int) ucnt && sm->stat_p[tid] == QHUFF_DEC_OK)
    {
        const QH_GLB uint32_t *gin_off = glb(a.in_off);
        const uint32_t o0 = gin_off[s0 + tid], o1 = gin_off[s0 + tid + 1];
        const uintptr_t pa = (uintptr_t) (a.in + o0) & ~(uintptr_t) 3;
        const uint32_t rs = (uint32_t) ((uintptr_t) (a.in + o0) - pa);
        GlobalEmit em{a.out + base + sm->excl_p[tid], 0};
        decode_string(DecGlb{(const QH_GLB uint32_t *) pa}, 8 * rs,
                      8 * (rs + o1 - o0), sm->win, sm->sorted, sm->longc, em);
    }
    if (tid < (int) ucnt)
    {
        gout_off[s0 + tid] = (uint32_t) (base + sm->excl_p[tid]);
        gstat[s0 + tid] = sm->stat_p[tid];
    }
    if (df.last && df.tile == a.c.n_tiles - 1 && tid == 0)
        gout_off[a.n] = (uint32_t) (base + df.total);
    stamp(a.c, df.tile, 13);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 3))) void
qhuff_decode_kernel(DecArgs a)
{
    __shared__ DecSmem smem;
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_claim;           // tile after `next` (look-back wave)
    __shared__ uint32_t s_red;             // next unit's end (unit_vote)
    __shared__ unsigned long long s_acc;   // tile aggregate accumulator
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    QH_LDS uint32_t *red = (QH_LDS uint32_t *) &s_red;
    const int tid = threadIdx.x;
    const bool lbw = is_lb_wave();
    if (a.c.dbg & kDbgCensus)
    {
        census(a.c);
        return;
    }
    {
        const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) glb(a.win);
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
        for (int i = tid; i < kWinSize / 4; i += kBlock)
            sw[i] = gw[i];
        const QH_GLB uint16_t *gs = glb(a.sorted);
        sm->sorted[tid] = gs[tid];
        if (tid == 0)
        {
            sm->sorted[256] = gs[256];
            s_acc = 0;
            s_red = 1;
        }
        if (tid < 4 * kMaxLong)
            ((QH_LDS uint32_t *) sm->longc)[tid] =
                ((const uint32_t *) a.lp.l)[tid];
    }
    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    uint32_t tile, next;
    claim_first(a.c, &tile, &next);
    if (tile >= a.c.n_tiles)
        return;

    // prologue: offsets, first unit and its input
    Prefetch<kDecChunks> pf;
    uint32_t cnt = (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) tile * kTile);
    pf.load_offsets(gin_off, (uint64_t) tile * kTile, cnt);
    pf.store_offsets(sm->off[0], cnt);
    __syncthreads();
    unit_vote(a.in, sm->off[0], 0, cnt, kDecInCap, red);
    __syncthreads();
    uint32_t lo = 0, hi = s_red;
    Span sp0 = unit_span(a.in, sm->off[0], lo, hi, kDecInCap);
    uintptr_t sp_pa = sp0.pa;
    uint32_t sp_n16 = sp0.n16;
    uint32_t sp_staged = sp0.staged;
    if (sp_staged)
    {
        pf.load_chunks(sp_pa, sp_n16);
        pf.store_chunks<true>((QH_LDS u32x4 *) sm->in, sp_n16);
    }
    uint32_t cur = 0;
    uint32_t unit_off = 0;                        // bytes of earlier units
    int64_t known_tile = -1;                      // see look_back_wave()
    uint64_t known_incl = 0, tile_base = 0;
    bool pending = false;
    Deferred df = {0, 0, 0, 0, 0, 0, false, false};

    for (;;)
    {
        const QH_LDS uint32_t *off = sm->off[cur];
        const bool last = hi == cnt;              // this unit ends the tile
        const bool has_next = next < a.c.n_tiles;
        const bool more = !last || has_next;      // a next unit exists
        const uint32_t lo_n = last ? 0 : hi;
        const uint32_t cnt_n = !last ? cnt : has_next
            ? (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) next * kTile) : 0;
        uint32_t claimed = a.c.n_tiles;
        if (tid == kBlock - 64 && last && has_next)
            claimed = claim_tile(a.c, next);      // consumed after the codec
        if (threadIdx.x < 64)
        {
            stamp(a.c, tile, 0);
            stamp(a.c, tile, 1);
            stamp_value(a.c, tile, 15, blockIdx.x);
            stamp_value(a.c, tile, 8, ((uint64_t) lo << 32) | hi);
        }
        if (last && has_next)
            pf.load_offsets(gin_off, (uint64_t) next * kTile, cnt_n);
        if (tid == 0)
            s_red = lo_n + 1;

        // 1. sort + decode the unit into the arena; each wave adds its byte
        //    total to the tile aggregate as soon as its strings are done
        const uint32_t ucnt = hi - lo;
        uint32_t key = 0;
        if (tid < (int) ucnt)
            key = min((off[lo + tid + 1] - off[lo + tid]) >> 1,
                      (uint32_t) kBuckets - 1);
        const uint32_t my = sort_by_bucket(key, sm->cnt, sm->perm);

        const bool valid = my < ucnt;
        const uint32_t A = off[lo];
        const uint32_t si = lo + (valid ? my : 0);
        const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (a.in + off[si]) - sp_pa) : 0;
        const uint32_t re = valid ? (uint32_t) ((uintptr_t) (a.in + off[si + 1]) - sp_pa) : 0;
        const uint32_t slot0 = 2 * my + (uint32_t) ((8ull * (off[si] - A)) / 5);
        uint32_t mine = 0;
        if (valid)
        {
            int r;
            if (a.c.dbg & kDbgNoCodec)
                r = (int) (re - rs);
            else if (sp_staged)
            {
                ArenaEmit em{sm->arena + slot0, 0};
                r = decode_string(DecLds{sm->in}, 8 * rs, 8 * re, sm->win,
                                  sm->sorted, sm->longc, em);
            }
            else
            {
                CountEmit em{0};
                r = decode_string(DecGlb{(const QH_GLB uint32_t *) sp_pa},
                                  8 * rs, 8 * re, sm->win, sm->sorted,
                                  sm->longc, em);
            }
            sm->size[my] = r < 0 ? 0x80000000u : (uint32_t) r;
            mine = r < 0 ? 0u : (uint32_t) r;
        }
        publish_wave_total(a.c, tile, mine, last,
                           (QH_LDS unsigned long long *) &s_acc);
        if (threadIdx.x < 64)
            stamp(a.c, tile, 2);
        else if (lbw)
            stamp(a.c, tile, 3);

        // look-back wave (shortest strings): the deferred unit's base
        if (lbw)
            stamp(a.c, tile, 5);
        if (pending && lbw)
        {
            const uint64_t b = resolve_unit_base(a.c, df, &known_tile,
                                                 &known_incl, &tile_base);
            if ((tid & 63) == 0)
                s_base = b;
        }
        if (tid == kBlock - 64)
            s_claim = claimed;
        if (lbw)
            stamp(a.c, tile, 6);
        if (last && has_next)
            pf.store_offsets(sm->off[cur ^ 1], cnt_n);
        __syncthreads();
        const uint32_t next2 = s_claim;
        if (threadIdx.x < 64)
            stamp(a.c, tile, 4);
        const QH_LDS uint32_t *off_n = last ? sm->off[cur ^ 1] : off;
        if (more)
            unit_vote(a.in, off_n, lo_n, cnt_n, kDecInCap, red);

        // 2. the deferred unit leaves: copy-out, offsets, status
        if (pending)
            finish_unit(a, sm, df, s_base);

        // 3. scan of this unit (its barrier also orders the copy-out reads
        //    above before the stage is cleared below, and the votes before
        //    the next unit's end is read); next unit's loads
        const uint32_t szw_t = tid < (int) ucnt ? sm->size[tid] : 0;
        const uint32_t sz_t = szw_t & 0x7fffffffu;
        uint32_t total;
        const uint32_t ex_t = block_excl_scan(sz_t, &sm->scr, &total);
        const uint32_t hi_n = s_red;
        uintptr_t nx_pa = 0;
        uint32_t nx_n16 = 0, nx_staged = 0;
        if (more)
        {
            Span t = unit_span(a.in, off_n, lo_n, hi_n, kDecInCap);
            nx_pa = t.pa;
            nx_n16 = t.n16;
            nx_staged = t.staged;
            if (nx_staged)
                pf.load_chunks(nx_pa, nx_n16);
        }

        // 4. compaction of this unit: arena slots -> output stage
        const bool staged_out = sp_staged && total + 64 <= (uint32_t) kDecOutCap;
        if (staged_out)
        {
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) sm->out;
            const uint32_t n16 = (total + 16 + 15) / 16 + 1;
            for (uint32_t i = tid; i < n16; i += kBlock)
                o4[i] = (u32x4){0, 0, 0, 0};
        }
        sm->excl_p[tid] = ex_t;
        sm->stat_p[tid] = (szw_t >> 31) ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
        __syncthreads();
        const uint32_t nout = valid ? sm->size[my] & 0x7fffffffu : 0;
        if (staged_out && nout && !(a.c.dbg & kDbgNoCodec))
        {
            const uint32_t D = 16 + sm->excl_p[my];
            const uint32_t dsh = 8 * (D & 3);
            const QH_LDS uint8_t *src = sm->arena + slot0;
            const uint32_t s3 = (uint32_t) ((uintptr_t) src & 3);
            const QH_LDS uint32_t *sw = (const QH_LDS uint32_t *) (src - s3);
            QH_LDS uint32_t *o = sm->out + (D >> 2);
            const uint32_t nwd = (nout + 3) >> 2;
            for (uint32_t k = 0; k < nwd; ++k)
            {
                uint32_t w = align_bytes(sw[k + 1], sw[k], s3);
                const uint32_t vb = nout - 4 * k;
                if (vb < 4)
                    w &= (1u << (8 * vb)) - 1;
                __hip_atomic_fetch_or(&o[k], w << dsh, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                if (dsh)
                    __hip_atomic_fetch_or(&o[k + 1], w >> (32 - dsh),
                                          __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        df.tile = tile;
        df.lo = lo;
        df.hi = hi;
        df.total = total;
        df.unit_off = unit_off;
        df.staged_out = staged_out;
        df.first = lo == 0;
        df.last = last;
        pending = true;
        unit_off = last ? 0 : unit_off + total;
        __syncthreads();
        if (threadIdx.x < 64)
            stamp(a.c, tile, 7);
        if (!more)
            break;
        if (nx_staged)
            pf.store_chunks<true>((QH_LDS u32x4 *) sm->in, nx_n16);
        if (last)
        {
            tile = next;
            next = next2;
            cnt = cnt_n;
            cur ^= 1;
        }
        lo = lo_n;
        hi = hi_n;
        sp_pa = nx_pa;
        sp_n16 = nx_n16;
        sp_staged = nx_staged;
    }
    if (lbw)
    {
        const uint64_t b = resolve_unit_base(a.c, df, &known_tile, &known_incl,
                                             &tile_base);
        if ((tid & 63) == 0)
            s_base = b;
    }
    __syncthreads();
    finish_unit(a, sm, df, s_base);
}

hipError_t
launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_decode_kernel, dim3(grid), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t
decode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_decode_kernel),
        kBlock, 0);
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
