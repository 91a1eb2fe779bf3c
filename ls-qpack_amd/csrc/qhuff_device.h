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
constexpr uint32_t kDbgCensus = 0x100;      // residency census only (below)
constexpr uint32_t kDbgStatic = 0x200;      // static tile order (needs the
                                            // whole grid resident)

// error bits reported through Coord::err
constexpr uint32_t kErrSpin = 1;            // look-back spin limit hit

struct Coord
{
    unsigned long long *flags;              // per-tile look-back flags
    uint32_t *err;                          // sticky device error word
    uint32_t *ctr;                          // claim counters [2][kGroups], strided
    uint32_t epoch;                         // launch tag carried in flags
    uint32_t n_tiles;
    uint32_t dbg;
    unsigned long long *trace;              // QHUFF_TRACE: kTraceSlots per tile
};

constexpr int kTraceSlots = 16;

// phase stamps for tools/trace_report.py (null trace: one scalar branch)
__device__ __forceinline__ void
stamp(const Coord &c, uint32_t tile, int slot)
{
    if (c.trace && (threadIdx.x & 63) == 0)
        c.trace[(uint64_t) kTraceSlots * tile + slot] =
            slot == 0 ? __builtin_amdgcn_s_memrealtime()
                      : __builtin_amdgcn_s_memtime();
}

__device__ __forceinline__ void
stamp_value(const Coord &c, uint32_t tile, int slot, uint64_t v)
{
    if (c.trace && (threadIdx.x & 63) == 0)
        c.trace[(uint64_t) kTraceSlots * tile + slot] = v;
}

struct LdsScratch                           // per-WG scan scratch
{
    uint32_t wsum[4];
};

// A workgroup is four waves, one string per lane (kBlock == kTile).  Every
// wave decodes/encodes; wave 3 (the "look-back wave") also claims tiles and
// resolves the decoupled look-back.  Tile aggregates are published by
// whichever wave finishes its strings last (publish_wave_total), so a
// tile's aggregate never waits for any look-back -- look-back waits cannot
// chain from one workgroup to the next.  Copy-out of the deferred tile is
// shared by all four waves.
constexpr int kBlock = kTile;
constexpr int kLoadThreads = kTile;
__device__ __forceinline__ bool
is_lb_wave()
{
    return threadIdx.x >= kTile - 64;
}

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
// Returns the tile-local string index this thread should process.  Waves
// take 64-string runs of the sorted order; the look-back wave (wave 3),
// which also resolves the look-back, takes the shortest run.
__device__ __forceinline__ uint32_t
sort_by_bucket(uint32_t key, QH_LDS uint32_t *s_cnt, QH_LDS uint16_t *s_perm)
{
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < kBuckets)
        s_cnt[tid] = 0;
    __syncthreads();
    const uint32_t pos = __hip_atomic_fetch_add(&s_cnt[key], 1u, __ATOMIC_RELAXED,
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
    return s_perm[(tid + 64) & (kTile - 1)];
}

// Look-back by ONE wave (the look-back wave):
// kLbK flags per lane, kLbWin predecessors per poll.  Position q of the
// window (q = 64k + lane) is tile j - q.
constexpr int kLbK = 12;
constexpr int kLbWin = kLbK * 64;

// known_tile / known_incl: a predecessor whose inclusive prefix the calling
// workgroup already knows (its own previous tile), or known_tile = -1.  With
// gridDim.x <= kLbWin one poll always reaches it.  Returns the exclusive
// byte prefix of `tile` and publishes its inclusive value (lane 0).
__device__ __forceinline__ uint64_t
look_back_wave(const Coord &c, uint32_t tile, uint64_t agg,
               int64_t known_tile, uint64_t known_incl, uint32_t *polls = nullptr,
               bool publish = true)
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
            if (++spins > ((c.dbg & kDbgStatic) ? (1u << 12) : kSpinLimit))
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
    if (lane == 0 && publish)
        __hip_atomic_store(&c.flags[tile],
                           kFlagInc | ep | ((excl + agg) & kValMask),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (polls)
        *polls = spins;
    return excl;
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
unit_span(const uint8_t *in, const QH_LDS uint32_t *s_off, uint32_t lo,
          uint32_t hi, uint32_t cap)
{
    Span sp;
    const uintptr_t a = (uintptr_t) (in + s_off[lo]);
    const uintptr_t b = (uintptr_t) (in + s_off[hi]);
    sp.pa = a & ~(uintptr_t) 15;
    const uintptr_t pb = (b + 15) & ~(uintptr_t) 15;
    sp.n16 = (uint32_t) ((pb - sp.pa) >> 4);
    sp.staged = pb - sp.pa <= (uintptr_t) cap;
    return sp;
}

// Units.  A tile's strings are coded in one or more consecutive units by the
// workgroup that claimed it: a unit is the longest run of the tile's
// remaining strings whose input fits the LDS stage (at least one string; a
// single string longer than the stage is read from global memory).  With
// header-sized strings a tile is one unit; the split keeps an oversized
// tile from taking a slow path that would stall every look-back behind it.
//
// unit_vote: every thread votes for one candidate end (tid + 1); the unit
// end is the largest candidate whose span fits.  *s_red must hold lo + 1
// before the votes; read it after a barrier.
__device__ __forceinline__ void
unit_vote(const uint8_t *in, const QH_LDS uint32_t *s_off, uint32_t lo,
          uint32_t cnt, uint32_t cap, QH_LDS uint32_t *s_red)
{
    const uint32_t j = threadIdx.x + 1;
    bool fits = false;
    if (j > lo + 1 && j <= cnt)
    {
        const uintptr_t pa = (uintptr_t) (in + s_off[lo]) & ~(uintptr_t) 15;
        const uintptr_t pb = ((uintptr_t) (in + s_off[j]) + 15) & ~(uintptr_t) 15;
        fits = pb - pa <= (uintptr_t) cap;
    }
    // fits is monotone in j: one LDS atomic per wave, for its last fit
    const uint64_t m = __ballot(fits);
    if (m && (threadIdx.x & 63) == 0)
        __hip_atomic_fetch_max(s_red, (threadIdx.x & ~63u) + 64 - __builtin_clzll(m),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Residency census (diagnostic launch, kDbgCensus): every workgroup counts
// itself in (arrivals, live), waits (bounded) until the whole grid has
// arrived, then counts itself out.  The peak of `live` is the number of
// workgroups that were on the device together.  Words: err[1] live,
// err[2] peak, err[3] arrivals.
__device__ __forceinline__ void
census(const Coord &c)
{
    if (threadIdx.x != 0)
        return;
    const uint32_t live = __hip_atomic_fetch_add(&c.err[1], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) + 1;
    __hip_atomic_fetch_max(&c.err[2], live, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    uint32_t v = __hip_atomic_fetch_add(&c.err[3], 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) + 1;
    for (uint32_t spins = 0; v < gridDim.x && spins < (1u << 14); ++spins)
    {
        __builtin_amdgcn_s_sleep(2);
        v = __hip_atomic_load(&c.err[3], __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_fetch_sub(&c.err[1], 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Dynamic tile order.  Workgroups form kGroups groups (blockIdx mod
// kGroups); group g owns tiles g, g + NG, g + 2 NG, ... (NG = min(kGroups,
// grid)) and its workgroups claim them in order from the group's counter.
// A look-back then only waits on tiles that a running workgroup holds or
// that its group will claim next, as long as every group has a running
// workgroup -- not that the whole grid is resident.  Spreading the claims
// over kGroups counters keeps same-address atomics from serialising.
// Launch `epoch` uses counter set epoch & 1 and clears the other set for
// the next launch on the stream (a context's launches are stream-ordered).
constexpr uint32_t kGroups = 64;
constexpr uint32_t kCtrStride = 64;        // u32 per counter: 256 B apart, so
                                           // groups never share a cache line

__device__ __forceinline__ uint32_t
claim_tile(const Coord &c, uint32_t prev)
{
    if (c.dbg & kDbgStatic)
    {
        const uint64_t t = (uint64_t) prev + gridDim.x;
        return t < c.n_tiles ? (uint32_t) t : c.n_tiles;
    }
    const uint32_t ng = gridDim.x < kGroups ? gridDim.x : kGroups;
    const uint32_t g = blockIdx.x % ng;
    const uint32_t k = __hip_atomic_fetch_add(
        &c.ctr[((c.epoch & 1) * kGroups + g) * kCtrStride], 1u,
        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t = g + (uint64_t) k * ng;
    return t < c.n_tiles ? (uint32_t) t : c.n_tiles;
}

// prologue: the first two tiles of this workgroup (every thread calls it)
__device__ __forceinline__ void
claim_first(const Coord &c, uint32_t *tile, uint32_t *next)
{
    __shared__ uint32_t s_pro[2];
    if (blockIdx.x == 0 && threadIdx.x < kGroups)
        __hip_atomic_store(
            &c.ctr[(((c.epoch + 1) & 1) * kGroups + threadIdx.x) * kCtrStride],
            0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0)
    {
        const uint32_t a = (c.dbg & kDbgStatic) ? blockIdx.x : claim_tile(c, 0);
        const uint32_t b = claim_tile(c, a);
        s_pro[0] = a < b ? a : b;
        s_pro[1] = a < b ? b : a;
    }
    __syncthreads();
    *tile = s_pro[0];
    *next = s_pro[1];
}

// Each wave adds its strings' total output bytes to the tile accumulator
// (wave count in [63:56], bytes below).  The wave that completes the count
// of the tile's LAST unit publishes the tile aggregate and clears the
// accumulator; after an earlier unit it only clears the count (bytes carry
// over).  Read again only after barriers.  Once per wave, all lanes active.
__device__ __forceinline__ void
publish_wave_total(const Coord &c, uint32_t tile, uint32_t my_bytes,
                   bool last_unit, QH_LDS unsigned long long *s_acc)
{
    uint64_t v = my_bytes;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        v += __shfl_xor(v, d, 64);
    if ((threadIdx.x & 63) == 0)
    {
        const uint64_t inc = (1ull << 56) + v;
        const uint64_t old = __hip_atomic_fetch_add(s_acc, inc, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((old >> 56) == (uint64_t) (kBlock / 64 - 1))
        {
            const uint64_t agg = (old + inc) & ((1ull << 56) - 1);
            *s_acc = last_unit ? 0 : agg;
            if (last_unit)
                __hip_atomic_store(&c.flags[tile],
                                   kFlagAgg | ((uint64_t) c.epoch << 40)
                                            | (agg & kValMask),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Copy `total` bytes that sit at LDS byte offset 16 (s_stage has 16 bytes of
// pad in front) to global `dst` (any alignment) with 16-byte aligned stores;
// the partial first/last 16-byte chunks are written byte by byte.  Called by
// every thread of the block.
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
    for (uint32_t k = threadIdx.x; k < nchunk; k += kBlock)
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
