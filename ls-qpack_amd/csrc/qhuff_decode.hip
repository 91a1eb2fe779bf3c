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
long_code(uint32_t w, const LongParams &lp, const QH_LDS uint16_t *s_sorted,
          uint32_t *len)
{
    uint32_t L = 0, idx = 0;
#pragma unroll
    for (int i = 0; i < kMaxLong; ++i)
    {
        // lengths past lp.n are padded with count 0 (never hit)
        uint32_t v = w >> (32 - lp.l[i].len);
        uint32_t off = v - lp.l[i].first;
        bool hit = (L == 0) & (off < lp.l[i].count);
        L = hit ? lp.l[i].len : L;
        idx = hit ? lp.l[i].base + off : idx;
    }
    *len = L;
    return s_sorted[idx];
}

// Decode one string whose bits are [bit0, bitend) of the big-endian dword
// stream `src`; emitted bytes go through `emit`.  Returns the number of
// output bytes, or -1 for a rejected string.  Loops are wave-uniform with
// the per-lane body under one predicate.
template <class Src, class Emit>
__device__ __forceinline__ int
decode_string(const Src &src, uint32_t bit0, uint32_t bitend,
              const QH_LDS uint32_t *s_win, const QH_LDS uint16_t *s_sorted,
              const LongParams &lp, Emit &emit)
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
    int nout = 0;
    bool bad = false;

    // main phase: >= 32 real bits ahead, no padding, no tail.  Invariant:
    // the buffer holds >= 32 valid bits and ends on a dword boundary (p).
    while (__builtin_amdgcn_ballot_w64(rem >= 32 && !bad))
    {
        if (rem >= 32 && !bad)
        {
            const uint32_t d = src.dw_ahead(p, bitend);   // refill candidate
            const uint32_t e = s_win[hi >> (32 - kWinBits)];
            const uint32_t ns = e >> 24;
            uint32_t c = (ns == 2) ? (e >> 20) & 15 : (e >> 16) & 15;
            uint32_t val = e;
            uint32_t nb = ns == 2 ? 2 : 1;
            if (__builtin_amdgcn_ballot_w64(ns == 0))
            {
                uint32_t L;
                const uint32_t sym = long_code(hi, lp, s_sorted, &L);
                c = ns == 0 ? L : c;
                val = ns == 0 ? sym : val;
                bad = (ns == 0) & (sym == 256);          // EOS in the data
                c = bad ? 0 : c;
                nb = bad ? 0 : nb;
            }
            emit(val, nb);
            nout += (int) nb;
            const uint32_t sh = __builtin_amdgcn_alignbit(hi, lo, (32 - c) & 31);
            hi = c ? sh : hi;
            lo = lo << (c & 31);
            bits -= c;
            rem -= c;
            const bool need = bits < 32;
            hi |= need ? d >> (bits & 31) : 0u;
            lo |= need ? d << ((32 - bits) & 31) : 0u;
            p += need ? 1 : 0;
            bits += need ? 32 : 0;
        }
    }

    // epilogue: the last < 32 bits, padded with ones; D3 tail rule
    bool fin = bad || rem == 0;
    while (__builtin_amdgcn_ballot_w64(!fin))
    {
        if (!fin)
        {
            const uint32_t w = hi | (0xffffffffu >> (rem & 31));
            const uint32_t e = s_win[w >> (32 - kWinBits)];
            const uint32_t ns = e >> 24, l0 = (e >> 16) & 15,
                           lt = (e >> 20) & 15;
            const bool two = (ns == 2) & (lt <= rem);
            uint32_t c = two ? lt : (ns ? l0 : 31u);
            uint32_t val = e;
            bool eos = false;
            if (__builtin_amdgcn_ballot_w64((ns == 0) & (rem > kWinBits)))
            {
                uint32_t L;
                const uint32_t sym = long_code(w, lp, s_sorted, &L);
                const bool lng = (ns == 0) & (rem > kWinBits);
                c = lng ? L : c;
                val = lng ? sym : val;
                eos = lng & (sym == 256);
            }
            if (c > rem)
            {
                // at most 7 bits of EOS prefix may remain
                const uint32_t ones = 0xffffffffu >> (32 - rem);
                bad = rem >= 8 || (w >> (32 - rem)) != ones;
                fin = true;
            }
            else if (eos)
            {
                bad = true;
                fin = true;
            }
            else
            {
                const uint32_t nb = two ? 2 : 1;
                emit(val, nb);
                nout += (int) nb;
                const uint32_t sh = __builtin_amdgcn_alignbit(hi, lo, (32 - c) & 31);
                hi = sh;                          // 5 <= c < 32 here
                lo = lo << c;
                rem -= c;
                fin = rem == 0;
            }
        }
    }
    return bad ? -1 : nout;
}

// byte-granular arena sink: two unconditional byte stores per step (the
// second is overwritten by the next step when only one symbol was emitted)
struct ArenaEmit
{
    QH_LDS uint8_t *slot;
    uint32_t pos;
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        slot[pos] = (uint8_t) val;
        slot[pos + 1] = (uint8_t) (val >> 8);
        pos += nb;
    }
};

struct CountEmit
{
    __device__ __forceinline__ void operator()(uint32_t, uint32_t) {}
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

// the tile whose look-back / copy-out is deferred to the next iteration
struct Deferred
{
    uint32_t tile, cnt, total;
    uint32_t staged_out;       // output sits in sm->out (else re-decode)
};

// look-back + copy-out + offsets of the deferred tile: store wave only
__device__ __forceinline__ void
finish_tile(const DecArgs &a, QH_LDS DecSmem *sm, const Deferred &df,
            int64_t *known_tile, uint64_t *known_incl)
{
    const int lane = threadIdx.x & 63;
    const uint64_t base = (a.c.dbg & kDbgNoLookback) ? (uint64_t) df.tile << 16
        : look_back_wave(a.c, df.tile, df.total, *known_tile, *known_incl);
    *known_tile = df.tile;
    *known_incl = base + df.total;
    if (a.c.dbg & kDbgNoStore)
        return;
    const uint64_t s0 = (uint64_t) df.tile * kTile;
    QH_GLB uint32_t *gout_off = glb(a.out_off);
    QH_GLB uint8_t *gstat = glb(a.status);
    if (df.staged_out)
        copy_out(sm->out, a.out + base, df.total);
    for (int t = lane; t < (int) df.cnt; t += 64)
    {
        gout_off[s0 + t] = (uint32_t) (base + sm->excl_p[t]);
        gstat[s0 + t] = sm->stat_p[t];
    }
    if (df.tile == a.c.n_tiles - 1 && lane == 0)
        gout_off[a.n] = (uint32_t) (base + df.total);
}

// slow path of a deferred tile whose output did not fit the LDS stage: every
// lane decodes its string again straight to global memory (input read from
// global).  Needs the tile base, which the store wave left in *s_base.
__device__ __forceinline__ void
finish_tile_slow(const DecArgs &a, QH_LDS DecSmem *sm, const Deferred &df,
                 uint64_t base)
{
    const int tid = threadIdx.x;
    if ((a.c.dbg & kDbgNoStore) || tid >= (int) df.cnt
            || sm->stat_p[tid] != QHUFF_DEC_OK)
        return;
    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    const uint64_t s0 = (uint64_t) df.tile * kTile;
    const uint32_t o0 = gin_off[s0 + tid], o1 = gin_off[s0 + tid + 1];
    const uintptr_t pa = (uintptr_t) (a.in + o0) & ~(uintptr_t) 3;
    const uint32_t rs = (uint32_t) ((uintptr_t) (a.in + o0) - pa);
    GlobalEmit em{a.out + base + sm->excl_p[tid], 0};
    decode_string(DecGlb{(const QH_GLB uint32_t *) pa}, 8 * rs,
                  8 * (rs + o1 - o0), sm->win, sm->sorted, a.lp, em);
}

__global__ __launch_bounds__(kTile) void
qhuff_decode_kernel(DecArgs a)
{
    __shared__ DecSmem smem;
    __shared__ uint64_t s_base;
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    const int tid = threadIdx.x;
    const bool ldw = !is_store_wave();
    {
        const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) glb(a.win);
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
        for (int i = tid; i < kWinSize / 4; i += kTile)
            sw[i] = gw[i];
        const QH_GLB uint16_t *gs = glb(a.sorted);
        sm->sorted[tid] = gs[tid];
        if (tid == 0)
            sm->sorted[256] = gs[256];
    }
    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    const uint32_t G = gridDim.x;
    uint32_t tile = blockIdx.x;
    if (tile >= a.c.n_tiles)
        return;

    // prologue: offsets + input of the first tile (load waves)
    Prefetch<kDecChunks> pf;
    uint32_t cnt = (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) tile * kTile);
    if (ldw)
    {
        pf.load_offsets(gin_off, (uint64_t) tile * kTile, cnt);
        pf.store_offsets(sm->off[0], cnt);
    }
    __syncthreads();
    Span sp0 = tile_span(a.in, sm->off[0], cnt, kDecInCap);
    uintptr_t sp_pa = sp0.pa;
    uint32_t sp_n16 = sp0.n16;
    uint32_t sp_staged = sp0.staged;
    if (sp_staged && ldw)
    {
        pf.load_chunks(sp_pa, sp_n16);
        pf.store_chunks<true>((QH_LDS u32x4 *) sm->in, sp_n16);
    }
    uint32_t cur = 0;
    int64_t known_tile = -1;                      // see look_back_wave()
    uint64_t known_incl = 0;
    bool pending = false;
    Deferred df = {0, 0, 0, 0};

    for (;;)
    {
        const QH_LDS uint32_t *off = sm->off[cur];
        const uint32_t next = tile + G;
        const bool has_next = next < a.c.n_tiles;
        const uint32_t cnt_n = has_next
            ? (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) next * kTile) : 0;
        if (threadIdx.x < 64)
        {
            stamp(a.c, tile, 0);
            stamp(a.c, tile, 1);
        }
        if (has_next && ldw)
            pf.load_offsets(gin_off, (uint64_t) next * kTile, cnt_n);

        // 1. sort + decode into the arena (sizes)
        uint32_t key = 0;
        if (tid < (int) cnt)
            key = min((off[tid + 1] - off[tid]) >> 1, (uint32_t) kBuckets - 1);
        const uint32_t my = sort_by_bucket(key, sm->cnt, sm->perm);
        const bool valid = my < cnt;
        const uint32_t A = off[0];
        const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (a.in + off[my]) - sp_pa) : 0;
        const uint32_t re = valid ? (uint32_t) ((uintptr_t) (a.in + off[my + 1]) - sp_pa) : 0;
        const uint32_t slot0 = 2 * my + (uint32_t) ((8ull * (off[my] - A)) / 5);
        if (valid)
        {
            int r;
            if (a.c.dbg & kDbgNoCodec)
                r = (int) (re - rs);
            else if (sp_staged)
            {
                ArenaEmit em{sm->arena + slot0, 0};
                r = decode_string(DecLds{sm->in}, 8 * rs, 8 * re, sm->win,
                                  sm->sorted, a.lp, em);
            }
            else
            {
                CountEmit em;
                r = decode_string(DecGlb{(const QH_GLB uint32_t *) sp_pa},
                                  8 * rs, 8 * re, sm->win, sm->sorted, a.lp, em);
            }
            sm->size[my] = r < 0 ? 0x80000000u : (uint32_t) r;
        }
        if (threadIdx.x < 64)
            stamp(a.c, tile, 2);
        else if (!ldw)
            stamp(a.c, tile, 3);
        if (has_next && ldw)
            pf.store_offsets(sm->off[cur ^ 1], cnt_n);
        __syncthreads();
        if (threadIdx.x < 64)
            stamp(a.c, tile, 4);

        // 2. scan
        const uint32_t szw_t = tid < (int) cnt ? sm->size[tid] : 0;
        const uint32_t sz_t = szw_t & 0x7fffffffu;
        uint32_t total;
        const uint32_t ex_t = block_excl_scan(sz_t, &sm->scr, &total);

        // 3. load waves: next tile's input loads (landed at the end);
        //    store wave: the deferred tile's look-back, copy-out, offsets,
        //    then this tile's aggregate
        uintptr_t nx_pa = 0;
        uint32_t nx_n16 = 0, nx_staged = 0;
        if (has_next)
        {
            Span t = tile_span(a.in, sm->off[cur ^ 1], cnt_n, kDecInCap);
            nx_pa = t.pa;
            nx_n16 = t.n16;
            nx_staged = t.staged;
            if (nx_staged && ldw)
                pf.load_chunks(nx_pa, nx_n16);
        }
        if (!ldw)
            stamp(a.c, tile, 5);
        if (pending && !ldw)
        {
            finish_tile(a, sm, df, &known_tile, &known_incl);
            if (!df.staged_out && (tid & 63) == 0)
                s_base = known_incl - df.total;
        }
        if (!ldw)
        {
            publish_aggregate(a.c, tile, total);
            stamp(a.c, tile, 6);
        }
        __syncthreads();
        if (pending && !df.staged_out)
            finish_tile_slow(a, sm, df, s_base);

        // 4. compaction of this tile: arena slots -> output stage
        const bool staged_out = sp_staged && total + 64 <= (uint32_t) kDecOutCap;
        if (staged_out)
        {
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) sm->out;
            const uint32_t n16 = (total + 16 + 15) / 16 + 1;
            for (uint32_t i = tid; i < n16; i += kTile)
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
        df.cnt = cnt;
        df.total = total;
        df.staged_out = staged_out;
        pending = true;
        __syncthreads();
        if (threadIdx.x < 64)
            stamp(a.c, tile, 7);
        if (!has_next)
            break;
        if (nx_staged && ldw)
            pf.store_chunks<true>((QH_LDS u32x4 *) sm->in, nx_n16);
        tile = next;
        cnt = cnt_n;
        sp_pa = nx_pa;
        sp_n16 = nx_n16;
        sp_staged = nx_staged;
        cur ^= 1;
    }
    if (!ldw)
    {
        finish_tile(a, sm, df, &known_tile, &known_incl);
        if ((tid & 63) == 0)
            s_base = known_incl - df.total;
    }
    __syncthreads();
    if (!df.staged_out)
        finish_tile_slow(a, sm, df, s_base);
}

hipError_t
launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_decode_kernel, dim3(grid), dim3(kTile), 0, st, a);
    return hipGetLastError();
}

hipError_t
decode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_decode_kernel),
        kTile, 0);
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
