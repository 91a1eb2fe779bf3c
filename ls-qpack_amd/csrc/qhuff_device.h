// qhuff_device.h -- device-side building blocks shared by the encode and
// decode kernels (gfx950, wave64).
//
// Execution model ("wave tiles"): a workgroup only exists to share one copy
// of the static code tables in LDS.  After the single table-load barrier
// every wave is an independent worker with a private LDS region; it claims
// tiles of kWT = 64 strings (one string per lane), stages the tile's packed
// input, runs the per-lane codec, scans the 64 output sizes with cross-lane
// operations, resolves the tile's output base with a decoupled look-back
// over per-tile flags, and copies the compacted output out with 16-byte
// stores.  No workgroup barrier is ever taken inside the tile loop, so the
// latency of one wave's loads / look-back polls hides under the codec work
// of the other waves on its SIMD.
//
//   * explicit LDS / global address spaces (a generic pointer into LDS
//     compiles to flat_load with global-memory latency)
//   * wave scans, wave-level decoupled look-back with bounded spins
//   * grouped dynamic tile claims (no residency assumption)
//   * split copy-out: stage -> registers, then 16-byte aligned stores
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qhuff {

#define QH_LDS __attribute__((address_space(3)))
#define QH_GLB __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWT = 64;                     // strings per wave tile

// Look-back flag word: [63:42] launch epoch, [41:40] state (1 aggregate,
// 2 inclusive), [39:0] byte count.  Epoch on top: within a launch an
// inclusive flag compares above an aggregate one, and any flag of this
// launch above every stale one, so super-tile flags published by different
// waves use atomic max and are never downgraded.
constexpr uint64_t kFlagAgg = 1ull << 40;
constexpr uint64_t kFlagInc = 2ull << 40;
constexpr uint64_t kValMask = (1ull << 40) - 1;
constexpr uint32_t kEpochMask = (1u << 22) - 1;
constexpr uint32_t kSpinLimit = 1u << 21;   // polls before giving up (~1 s)
constexpr int kSuper = 64;                  // tiles per super tile
// super-tile accumulator word: [63:48] tiles arrived, [47:0] byte sum
constexpr uint64_t kAccOne = 1ull << 48;
constexpr uint64_t kAccMask = kAccOne - 1;

// ablation switches (timing experiments only; outputs are wrong when set)
constexpr uint32_t kDbgNoLookback = 2;      // base = tile * 8 KiB
constexpr uint32_t kDbgNoStore = 4;         // skip the global output stores
constexpr uint32_t kDbgNoCodec = 8;         // skip the per-string codec loops

constexpr uint32_t kDbgClock = 0x40;        // per-phase cycle sums (below)

// error bits reported through Coord::err
constexpr uint32_t kErrSpin = 1;            // look-back spin limit hit

// Dynamic tile order.  Waves form kGroups groups (global wave id mod
// kGroups); group g owns tiles g, g + NG, g + 2 NG, ... (NG = min(kGroups,
// waves)) and its waves claim them in order from the group's counter.  A
// tile is only ever claimed by a running wave, and every wave processes its
// claimed tiles in increasing order, so the lowest unfinished tile always
// makes progress: the look-back needs no residency guarantee.  Spreading the
// claims over kGroups counters keeps same-address atomics from serialising.
// Launch `epoch` uses counter set epoch & 1 and clears the other set for the
// next launch on the stream (a context's launches are stream-ordered).
constexpr uint32_t kGroups = 64;
constexpr uint32_t kCtrStride = 64;         // u32 per counter: 256 B apart

struct Coord
{
    unsigned long long *flags;              // per-tile look-back flags
    unsigned long long *sflags;             // per-super-tile flags
    unsigned long long *sacc;               // super accumulators [2][cap_super]
    uint32_t *err;                          // sticky device error word
    uint32_t *ctr;                          // claim counters [2][kGroups], strided
    uint32_t epoch;                         // launch tag carried in flags
    uint32_t n_tiles;
    uint32_t cap_super;                     // sacc entries per parity
    uint32_t dbg;
};

__device__ __forceinline__ uint32_t
lane_id()
{
    return threadIdx.x & 63;
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

__device__ __forceinline__ uint32_t
uniform(uint32_t v)
{
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t
read_lane(uint32_t v, uint32_t lane)
{
    return __builtin_amdgcn_readlane(v, lane);
}

// orders this wave's LDS accesses across lanes (LDS instructions of one
// wave execute in issue order; this stops the compiler moving them)
__device__ __forceinline__ void
wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wave inclusive scan of one uint32 per lane
__device__ __forceinline__ uint32_t
wave_incl_scan(uint32_t v)
{
    const uint32_t lane = lane_id();
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1)
    {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t) d ? y : 0u;
    }
    return x;
}

template <class T>
__device__ __forceinline__ T
wave_sum(T v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        v += __shfl_xor(v, d, 64);
    return v;
}

// Per-phase cycle accounting (kDbgClock): each wave sums s_memtime deltas
// per phase in registers and adds them once, at exit, to err[16 + 2 * ph]
// (u64 pairs).  Phase list: see the kernels.
constexpr int kPhases = 8;
struct PhaseClock
{
    uint64_t t0;
    uint64_t sum[kPhases];
    bool on;

    __device__ __forceinline__ void init(uint32_t dbg)
    {
        on = (dbg & kDbgClock) != 0;
        for (int i = 0; i < kPhases; ++i)
            sum[i] = 0;
        t0 = on ? __builtin_amdgcn_s_memtime() : 0;
    }
    __device__ __forceinline__ void lap(int ph)
    {
        if (on)
        {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            sum[ph] += t - t0;
            t0 = t;
        }
    }
    __device__ __forceinline__ void flush(uint32_t *err) const
    {
        if (on && (threadIdx.x & 63) == 0)
            for (int i = 0; i < kPhases; ++i)
                atomicAdd((unsigned long long *) (err + 16 + 2 * i),
                          (unsigned long long) sum[i]);
    }
};

// ---- tile claims -------------------------------------------------------

__device__ __forceinline__ uint32_t
wave_gid(int waves_per_block)
{
    return blockIdx.x * (uint32_t) waves_per_block + (threadIdx.x >> 6);
}

// lane 0 claims; the returned tile id is wave-uniform (n_tiles = none)
__device__ __forceinline__ uint32_t
claim_tile(const Coord &c, uint32_t gid, uint32_t n_waves)
{
    const uint32_t ng = n_waves < kGroups ? n_waves : kGroups;
    const uint32_t g = gid % ng;
    uint32_t k = 0;
    if (lane_id() == 0)
        k = __hip_atomic_fetch_add(
            &c.ctr[((c.epoch & 1) * kGroups + g) * kCtrStride], 1u,
            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    k = uniform(k);
    const uint64_t t = g + (uint64_t) k * ng;
    return t < c.n_tiles ? (uint32_t) t : c.n_tiles;
}

// clears the claim counters and super accumulators of the next launch on
// the stream (they use the other parity; every thread of the grid helps)
__device__ __forceinline__ void
clear_next_launch(const Coord &c)
{
    const uint32_t par = (c.epoch + 1) & 1;
    if (blockIdx.x == 0 && threadIdx.x < kGroups)
        __hip_atomic_store(&c.ctr[(par * kGroups + threadIdx.x) * kCtrStride],
                           0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // all of them: the next launch may hold more tiles than this one
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < c.cap_super;
         i += gridDim.x * blockDim.x)
        __hip_atomic_store(&c.sacc[(uint64_t) par * c.cap_super + i], 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- tile offsets ------------------------------------------------------

// Lane i holds the start offset of string i of the tile and of string i+1
// (clamped to the tile end).  `cnt` strings, cnt in [1, 64].
struct TileOffs
{
    uint32_t o0, o1;

    __device__ __forceinline__ void load(const QH_GLB uint32_t *in_off,
                                         uint64_t s0, uint32_t cnt)
    {
        const uint32_t lane = lane_id();
        o0 = in_off[s0 + (lane < cnt ? lane : cnt)];
        o1 = in_off[s0 + (lane + 1 < cnt ? lane + 1 : cnt)];
    }
    __device__ __forceinline__ uint32_t first() const { return read_lane(o0, 0); }
    __device__ __forceinline__ uint32_t last() const { return read_lane(o1, 63); }
};

// A tile's input span [pa, pb) rounded out to 16-byte boundaries.
struct Span
{
    uintptr_t pa;
    uint32_t n16;
    bool staged;
};

__device__ __forceinline__ Span
tile_span(const uint8_t *in, uint32_t A, uint32_t B, uint32_t cap)
{
    Span sp;
    const uintptr_t a = (uintptr_t) (in + A);
    const uintptr_t b = (uintptr_t) (in + B);
    sp.pa = a & ~(uintptr_t) 15;
    const uintptr_t pb = (b + 15) & ~(uintptr_t) 15;
    sp.n16 = (uint32_t) ((pb - sp.pa) >> 4);
    sp.staged = pb - sp.pa <= (uintptr_t) cap;
    return sp;
}

// A tile's staged input held in registers between its load and its LDS
// write: NCH 16-byte chunks per lane.
template <int NCH>
struct Chunks
{
    u32x4 ch[NCH];

    __device__ __forceinline__ void load(const Span &sp)
    {
        const uint32_t lane = lane_id();
#pragma unroll
        for (int k = 0; k < NCH; ++k)
        {
            const uint32_t i = lane + 64u * k;
            if (i < sp.n16)
                ch[k] = ((const QH_GLB u32x4 *) sp.pa)[i];
        }
    }
    template <bool SWAP>
    __device__ __forceinline__ void store(QH_LDS u32x4 *dst, uint32_t n16) const
    {
        const uint32_t lane = lane_id();
#pragma unroll
        for (int k = 0; k < NCH; ++k)
        {
            const uint32_t i = lane + 64u * k;
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

// ---- two-level decoupled look-back, one wave per tile ---------------------
//
// With thousands of waves each holding one tile, a flat look-back has to
// walk back through ~one tile per running wave before it meets an inclusive
// flag.  Tiles are therefore grouped into super tiles of kSuper consecutive
// tiles.  After its codec a tile publishes its aggregate and adds it to its
// super tile's accumulator; the tile whose add completes the count publishes
// the super tile's aggregate.  A tile's exclusive prefix is then
//   (aggregates of the earlier tiles of its super tile, back to an
//    inclusive one if there is one)
// + (super aggregates back to an inclusive super flag),
// one 64-wide window of each, polled together.  Only aggregates are waited
// for, and those are published right after codecs that are already running
// (tiles are claimed in order), so no wait chains through other look-backs.
// The last tile of a super tile publishes the super tile's inclusive flag.

__device__ __forceinline__ bool
flag_valid(uint64_t f, uint32_t epoch)
{
    return (f >> 42) == epoch && ((f >> 40) & 3) != 0;
}

__device__ __forceinline__ bool
flag_inc(uint64_t f)
{
    return ((f >> 40) & 3) == 2;
}

struct LookBack
{
    uint32_t tile, s;
    uint64_t total;
    uint64_t acc_old;            // returned by the super accumulator add (lane 0)
    uint64_t ft, fs;             // polled tile / super flags (one per lane)

    __device__ __forceinline__ uint64_t ep(const Coord &c) const
    {
        return (uint64_t) c.epoch << 42;
    }
    __device__ __forceinline__ void poll_tiles(const Coord &c)
    {
        const uint32_t lane = lane_id();
        const uint32_t f0 = s * kSuper;
        ft = (tile - f0 > lane) ? __hip_atomic_load(&c.flags[tile - 1 - lane],
                                                    __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : 0ull;
    }
    // super flags s-1-lane-64*back (before super 0: inclusive 0)
    __device__ __forceinline__ uint64_t poll_supers(const Coord &c,
                                                    uint32_t back) const
    {
        const int64_t j = (int64_t) s - 1 - lane_id() - 64 * (int64_t) back;
        return j < 0 ? (kFlagInc | ep(c))
                     : __hip_atomic_load(&c.sflags[j], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    }

    // publish the aggregate, add to the super accumulator, issue the polls
    __device__ __forceinline__ void start(const Coord &c, uint32_t t,
                                          uint64_t tot)
    {
        tile = t;
        s = t / kSuper;
        total = tot;
        acc_old = 0;
        if (lane_id() == 0)
        {
            __hip_atomic_store(&c.flags[t], kFlagAgg | ep(c) | (tot & kValMask),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc_old = __hip_atomic_fetch_add(
                &c.sacc[(uint64_t) (c.epoch & 1) * c.cap_super + s],
                kAccOne + tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        poll_tiles(c);
        fs = poll_supers(c, 0);
    }

    __device__ __forceinline__ void publish_super(const Coord &c, uint64_t state,
                                                  uint64_t v) const
    {
        if (lane_id() == 0)
            __hip_atomic_fetch_max(&c.sflags[s], state | ep(c) | (v & kValMask),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    __device__ __forceinline__ bool spin(const Coord &c, uint32_t *spins) const
    {
        if (++*spins > kSpinLimit)
        {
            if (lane_id() == 0)
                atomicOr(c.err, kErrSpin);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
        return true;
    }

    // returns the exclusive prefix of the tile; publishes its inclusive one
    __device__ __forceinline__ uint64_t finish(const Coord &c)
    {
        const uint32_t lane = lane_id();
        const uint32_t f0 = s * kSuper;
        const uint32_t in_super = c.n_tiles - f0 < (uint32_t) kSuper
                                ? c.n_tiles - f0 : (uint32_t) kSuper;
        // the add that completes the super tile publishes its aggregate
        const uint64_t old = ((uint64_t) read_lane((uint32_t) (acc_old >> 32), 0) << 32)
                           | read_lane((uint32_t) acc_old, 0);
        if ((old >> 48) == in_super - 1)
            publish_super(c, kFlagAgg, (old + total) & kAccMask);

        uint32_t spins = 0;
        uint64_t excl = 0;
        const uint32_t nq = tile - f0;               // earlier tiles in super
        // 1. earlier tiles of this super tile
        bool done = false;
        for (;;)
        {
            const bool inq = lane < nq;
            const uint64_t inv = __ballot(inq && !flag_valid(ft, c.epoch));
            const uint64_t inc = __ballot(inq && flag_valid(ft, c.epoch)
                                          && flag_inc(ft));
            const int F = inc ? __builtin_ctzll(inc) : 64;
            const uint64_t upto = F >= 63 ? ~0ull : ((2ull << F) - 1);
            if ((inv & upto) == 0)
            {
                excl = wave_sum((inq && (int) lane <= F) ? (ft & kValMask)
                                                         : 0ull);
                done = inc != 0;
                break;
            }
            if (!spin(c, &spins))
            {
                done = true;
                break;
            }
            poll_tiles(c);
        }
        // 2. super tiles before this one, back to an inclusive one
        for (uint32_t back = 0; !done;)
        {
            const uint64_t inv = __ballot(!flag_valid(fs, c.epoch));
            const uint64_t inc = __ballot(flag_valid(fs, c.epoch) && flag_inc(fs));
            const int G = inc ? __builtin_ctzll(inc) : 64;
            const uint64_t upto = G >= 63 ? ~0ull : ((2ull << G) - 1);
            if ((inv & upto) == 0)
            {
                excl += wave_sum((int) lane <= G ? (fs & kValMask) : 0ull);
                if (inc)
                    break;
                fs = poll_supers(c, ++back);
                continue;
            }
            if (!spin(c, &spins))
                break;
            fs = poll_supers(c, back);
        }
        if (lane == 0)
            __hip_atomic_store(&c.flags[tile],
                               kFlagInc | ep(c) | ((excl + total) & kValMask),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tile == f0 + in_super - 1)
            publish_super(c, kFlagInc, excl + total);
        return excl;
    }
};

// ---- copy-out -------------------------------------------------------------

// Copy of `total` bytes that sit at LDS byte offset 16 of a stage (16 bytes
// of pad in front, 32 bytes of readable slack behind) to global `dst` (any
// alignment), split so the stage can be refilled between reading it and
// storing: gather() reads every chunk this lane stores into registers,
// store() writes them (16-byte aligned stores; the partial first and last
// chunks byte by byte).  NCH chunks per lane cover 64 * NCH * 16 bytes.
template <int NCH>
struct CopyOut
{
    u32x4 o[NCH];
    uint8_t *g0;
    uint32_t r, nchunk, total;

    __device__ __forceinline__ void gather(const QH_LDS uint32_t *s_stage,
                                           uint8_t *dst, uint32_t tot)
    {
        total = tot;
        r = (uint32_t) ((uintptr_t) dst & 15);
        g0 = dst - r;                          // 16-byte aligned
        nchunk = tot ? (r + tot + 15) >> 4 : 0;
        // global chunk k holds stage bytes [16 + 16k - r, +16)
        const uint32_t sh = (16 - r) & 15;     // byte shift inside the stage
        const uint32_t c0 = (16 - r) >> 4;     // 1 when r == 0, else 0
        const uint32_t q = sh >> 2, bs = sh & 3;
        const QH_LDS uint32_t *s = s_stage + 4 * c0 + q;
        const uint32_t lane = lane_id();
#pragma unroll
        for (int j = 0; j < NCH; ++j)
        {
            const uint32_t k = lane + 64u * j;
            if (k < nchunk)
            {
                const QH_LDS uint32_t *p = s + 4 * k;
                const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3],
                               d4 = p[4];
                o[j] = (u32x4){align_bytes(d1, d0, bs), align_bytes(d2, d1, bs),
                               align_bytes(d3, d2, bs), align_bytes(d4, d3, bs)};
            }
        }
    }
    __device__ __forceinline__ void store() const
    {
        const uint32_t lane = lane_id();
#pragma unroll
        for (int j = 0; j < NCH; ++j)
        {
            const uint32_t k = lane + 64u * j;
            if (k < nchunk)
            {
                const uint32_t lo = k == 0 ? r : 0;
                const uint32_t hi = (k == nchunk - 1) ? r + total - 16 * k : 16;
                if (lo == 0 && hi == 16)
                    *(QH_GLB u32x4 *) (g0 + 16 * k) = o[j];
                else
                {
                    const u32x4 v = o[j];
                    for (uint32_t b = lo; b < hi; ++b)
                    {
                        const uint32_t qq = b >> 2;
                        const uint32_t wv = qq == 0 ? v.x : qq == 1 ? v.y
                                          : qq == 2 ? v.z : v.w;
                        ((QH_GLB uint8_t *) g0)[16 * k + b] =
                            (uint8_t) (wv >> (8 * (b & 3)));
                    }
                }
            }
        }
    }
};

}  // namespace qhuff
