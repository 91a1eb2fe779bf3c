// qhuff_device.h -- device-side building blocks shared by the encode and
// decode tile kernels (gfx950, wave64, 256-thread workgroups).
//
//   * explicit LDS / global address spaces (a generic pointer into LDS
//     compiles to flat_load with global-memory latency)
//   * workgroup exclusive scan
//   * length-bucket counting sort of a tile's strings, so that each wave runs
//     strings of similar length (the per-lane codec loops run as long as the
//     wave's longest string)
//   * 256-wide decoupled look-back over per-tile flags, with bounded spins
//   * shifted, 16-byte-aligned copy-out of an LDS output stage
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qhuff {

#define QH_LDS __attribute__((address_space(3)))
#define QH_GLB __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kTile = 256;                  // strings per tile = threads per WG
constexpr int kBuckets = 64;                // length buckets for the tile sort

// look-back flag word: [63:62] state, [61:40] epoch, [39:0] byte count
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 40) - 1;
constexpr uint32_t kEpochMask = (1u << 22) - 1;
constexpr uint32_t kSpinLimit = 1u << 21;   // polls before giving up (~1 s)

// ablation switches (timing experiments only; outputs are wrong when set)
constexpr uint32_t kDbgNoLookback = 2;      // base = tile * 64 KiB
constexpr uint32_t kDbgNoStore = 4;         // skip the global output stores
constexpr uint32_t kDbgNoCodec = 8;         // skip the per-string codec loops

// error bits reported through Coord::err
constexpr uint32_t kErrSpin = 1;            // look-back spin limit hit

struct Coord
{
    unsigned long long *flags;              // per-tile look-back flags
    uint32_t *err;                          // sticky device error word
    uint32_t epoch;                         // launch tag carried in flags
    uint32_t n_tiles;
    uint32_t dbg;
    unsigned long long *trace;              // QHUFF_TRACE: 8 stamps per tile
};

// phase stamps for tools/trace_report.py (null trace: one scalar branch)
__device__ __forceinline__ void
stamp(const Coord &c, uint32_t tile, int slot)
{
    if (c.trace && (threadIdx.x & 63) == 0)
        c.trace[8ull * tile + slot] = slot == 0 ? __builtin_amdgcn_s_memrealtime()
                                                : __builtin_amdgcn_s_memtime();
}

struct LdsScratch                           // per-WG scan scratch
{
    uint32_t wsum[4];
};

__device__ __forceinline__ uint32_t
bswap32(uint32_t v)
{
    return __builtin_bswap32(v);
}

// bytes [sh, sh+4) of the little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t
align_bytes(uint32_t hi, uint32_t lo, uint32_t sh)
{
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// workgroup exclusive scan of one uint32 per thread; *total = sum
__device__ __forceinline__ uint32_t
block_excl_scan(uint32_t v, QH_LDS LdsScratch *scr, uint32_t *total)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d)
            x += y;
    }
    if (lane == 63)
        scr->wsum[wave] = x;
    __syncthreads();
    uint32_t w0 = scr->wsum[0], w1 = scr->wsum[1], w2 = scr->wsum[2],
             w3 = scr->wsum[3];
    uint32_t before = (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0)
                    + (wave > 2 ? w2 : 0);
    *total = w0 + w1 + w2 + w3;
    return before + x - v;
}

// Counting sort of the tile's strings by length bucket (0..kBuckets-1).
// Returns the tile-local string index this thread should process.
__device__ __forceinline__ uint32_t
sort_by_bucket(uint32_t key, QH_LDS uint32_t *s_cnt, QH_LDS uint16_t *s_perm)
{
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < kBuckets)
        s_cnt[tid] = 0;
    __syncthreads();
    uint32_t pos = __hip_atomic_fetch_add(&s_cnt[key], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    if (tid < 64)
    {
        const uint32_t a = s_cnt[lane];
        uint32_t x = a;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1)
        {
            uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d)
                x += y;
        }
        s_cnt[lane] = x - a;
    }
    __syncthreads();
    s_perm[s_cnt[key] + pos] = (uint16_t) tid;
    __syncthreads();
    return s_perm[tid];
}

// Look-back by ONE wave (the store wave, see the kernels' role split):
// kLbK flags per lane, kLbWin predecessors per poll.  Position q of the
// window (q = 64k + lane) is tile j - q.
constexpr int kLbK = 16;
constexpr int kLbWin = kLbK * 64;

// known_tile / known_incl: a predecessor whose inclusive prefix the calling
// workgroup already knows (its own previous tile), or known_tile = -1.  With
// gridDim.x <= kLbWin one poll always reaches it.  Returns the exclusive
// byte prefix of `tile` and publishes its inclusive value (lane 0).
__device__ __forceinline__ uint64_t
look_back_wave(const Coord &c, uint32_t tile, uint64_t agg,
               int64_t known_tile, uint64_t known_incl)
{
    const int lane = threadIdx.x & 63;
    const uint64_t ep = (uint64_t) c.epoch << 40;
    uint64_t excl = 0;
    int64_t j = (int64_t) tile - 1;
    uint32_t spins = 0;
    while (j >= 0)
    {
        uint64_t f[kLbK];
#pragma unroll
        for (int k = 0; k < kLbK; ++k)
        {
            const int64_t idx = j - lane - 64 * k;
            if (idx < 0)
                f[k] = kFlagInc | ep;                    // before tile 0
            else if (idx == known_tile)
                f[k] = kFlagInc | ep | (known_incl & kValMask);
            else
                f[k] = __hip_atomic_load(&c.flags[idx], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
        int F = kLbWin;                  // nearest inclusive position
        uint64_t inv[kLbK];
#pragma unroll
        for (int k = kLbK - 1; k >= 0; --k)
        {
            const bool valid = ((f[k] >> 40) & kEpochMask) == c.epoch
                             && (f[k] >> 62) != 0;
            const bool inc = valid && (f[k] >> 62) == 2;
            const uint64_t im = __ballot(inc);
            inv[k] = __ballot(!valid);
            if (im)
                F = 64 * k + __builtin_ctzll(im);
        }
        const int fcap = F < kLbWin ? F : kLbWin - 1;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < kLbK; ++k)
        {
            const int lim = fcap - 64 * k;
            const uint64_t m = lim >= 63 ? ~0ull
                             : (lim < 0 ? 0ull : ((2ull << lim) - 1));
            bad |= (inv[k] & m) != 0;
        }
        if (bad)
        {
            if (++spins > kSpinLimit)
            {
                if (lane == 0)
                    atomicOr(c.err, kErrSpin);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t mine = 0;
#pragma unroll
        for (int k = 0; k < kLbK; ++k)
            mine += (lane + 64 * k <= F) ? (f[k] & kValMask) : 0;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1)
            mine += __shfl_xor(mine, d, 64);
        excl += mine;
        if (F < kLbWin)
            break;
        j -= kLbWin;
    }
    if (lane == 0)
        __hip_atomic_store(&c.flags[tile],
                           kFlagInc | ep | ((excl + agg) & kValMask),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// the store wave (wave 3) issues every global store and the look-back; the
// load waves (0..2) issue every prefetch load and never store, so their
// s_waitcnt vmcnt never drains a store (vmcnt counts loads and stores in
// issue order, MI355X_MICROARCH.md sec. per-instruction constants)
constexpr int kLoadThreads = 192;
__device__ __forceinline__ bool
is_store_wave()
{
    return threadIdx.x >= kLoadThreads;
}

// Next-tile prefetch: offsets and up to NCH 16-byte input chunks per thread
// held in registers while the current tile is processed.
template <int NCH>
struct Prefetch
{
    uint32_t off0, off1;            // two offsets per load thread (257 needed)
    u32x4 ch[NCH];

    __device__ __forceinline__ void load_offsets(const QH_GLB uint32_t *in_off,
                                                 uint64_t s0, uint32_t cnt)
    {
        const int tid = threadIdx.x;       // load waves only
        off0 = tid <= (int) cnt ? in_off[s0 + tid] : 0;
        const int t1 = tid + kLoadThreads;
        off1 = t1 <= (int) cnt ? in_off[s0 + t1] : 0;
    }
    __device__ __forceinline__ void store_offsets(QH_LDS uint32_t *s_off,
                                                  uint32_t cnt) const
    {
        const int tid = threadIdx.x;
        if (tid <= (int) cnt)
            s_off[tid] = off0;
        const int t1 = tid + kLoadThreads;
        if (t1 <= (int) cnt)
            s_off[t1] = off1;
    }
    __device__ __forceinline__ void load_chunks(uintptr_t pa, uint32_t n16)
    {
#pragma unroll
        for (int k = 0; k < NCH; ++k)
        {
            uint32_t i = threadIdx.x + k * kLoadThreads;
            if (i < n16)
                ch[k] = ((const QH_GLB u32x4 *) pa)[i];
        }
    }
    template <bool SWAP>
    __device__ __forceinline__ void store_chunks(QH_LDS u32x4 *dst,
                                                 uint32_t n16) const
    {
#pragma unroll
        for (int k = 0; k < NCH; ++k)
        {
            uint32_t i = threadIdx.x + k * kLoadThreads;
            if (i < n16)
            {
                u32x4 v = ch[k];
                if (SWAP)
                    v = (u32x4){bswap32(v.x), bswap32(v.y), bswap32(v.z),
                                bswap32(v.w)};
                dst[i] = v;
            }
        }
    }
};

// A tile's input span [pa, pb) rounded out to 16-byte boundaries.
struct Span
{
    uintptr_t pa;
    uint32_t n16;
    bool staged;
};

__device__ __forceinline__ Span
tile_span(const uint8_t *in, const QH_LDS uint32_t *s_off, uint32_t cnt,
          uint32_t cap)
{
    Span sp;
    const uintptr_t a = (uintptr_t) (in + s_off[0]);
    const uintptr_t b = (uintptr_t) (in + s_off[cnt]);
    sp.pa = a & ~(uintptr_t) 15;
    const uintptr_t pb = (b + 15) & ~(uintptr_t) 15;
    sp.n16 = (uint32_t) ((pb - sp.pa) >> 4);
    sp.staged = pb - sp.pa <= (uintptr_t) cap;
    return sp;
}

__device__ __forceinline__ void
publish_aggregate(const Coord &c, uint32_t tile, uint64_t agg)
{
    if (threadIdx.x == kLoadThreads)        // first lane of the store wave
        __hip_atomic_store(&c.flags[tile],
                           kFlagAgg | ((uint64_t) c.epoch << 40)
                           | (agg & kValMask),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Copy `total` bytes that sit at LDS byte offset 16 (s_stage has 16 bytes of
// pad in front) to global `dst` (any alignment) with 16-byte aligned stores;
// the partial first/last 16-byte chunks are written byte by byte.  Called by
// the store wave (64 lanes).
__device__ __forceinline__ void
copy_out(const QH_LDS uint32_t *s_stage, uint8_t *dst, uint32_t total)
{
    if (total == 0)
        return;
    const uint32_t r = (uint32_t) ((uintptr_t) dst & 15);
    uint8_t *g0 = dst - r;                   // 16-byte aligned
    const uint32_t nchunk = (r + total + 15) >> 4;
    // global chunk k holds stage bytes [16 + 16k - r, +16)
    const uint32_t sh = (16 - r) & 15;       // byte shift inside the stage
    const uint32_t c0 = (16 - r) >> 4;       // 1 when r == 0, else 0
    const QH_LDS u32x4 *s4 = (const QH_LDS u32x4 *) s_stage;
    for (uint32_t k = threadIdx.x & 63; k < nchunk; k += 64)
    {
        u32x4 a = s4[k + c0], b = s4[k + c0 + 1];
        uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t q = sh >> 2, bs = sh & 3;
        u32x4 o;
        // q is uniform across the workgroup
        switch (q)
        {
        case 0: o = (u32x4){align_bytes(d[1], d[0], bs), align_bytes(d[2], d[1], bs),
                            align_bytes(d[3], d[2], bs), align_bytes(d[4], d[3], bs)}; break;
        case 1: o = (u32x4){align_bytes(d[2], d[1], bs), align_bytes(d[3], d[2], bs),
                            align_bytes(d[4], d[3], bs), align_bytes(d[5], d[4], bs)}; break;
        case 2: o = (u32x4){align_bytes(d[3], d[2], bs), align_bytes(d[4], d[3], bs),
                            align_bytes(d[5], d[4], bs), align_bytes(d[6], d[5], bs)}; break;
        default: o = (u32x4){align_bytes(d[4], d[3], bs), align_bytes(d[5], d[4], bs),
                             align_bytes(d[6], d[5], bs), align_bytes(d[7], d[6], bs)}; break;
        }
        const uint32_t lo = k == 0 ? r : 0;
        const uint32_t hi = (k == nchunk - 1) ? r + total - 16 * k : 16;
        if (lo == 0 && hi == 16)
            *(QH_GLB u32x4 *) (g0 + 16 * k) = o;
        else
        {
            for (uint32_t b2 = lo; b2 < hi; ++b2)
            {
                uint32_t q2 = b2 >> 2;
                uint32_t wv = q2 == 0 ? o.x : q2 == 1 ? o.y : q2 == 2 ? o.z : o.w;
                g0[16 * k + b2] = (uint8_t) (wv >> (8 * (b2 & 3)));
            }
        }
    }
}

}  // namespace qhuff
