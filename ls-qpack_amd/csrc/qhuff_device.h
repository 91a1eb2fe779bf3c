// qhuff_device.h -- device-side building blocks shared by the encode and
// decode kernels (gfx950, wave64).
//
// Execution model ("wave tiles"): a workgroup only exists to share one copy
// of the static code tables in LDS.  After the single table-load barrier
// every wave is an independent worker with a private LDS region; it codes
// tiles of kWT = 64 strings (one string per lane), scans the 64 output sizes
// with cross-lane operations, resolves each tile's output base with a
// two-level decoupled look-back and stores the compacted output with 16-byte
// stores.  No workgroup barrier is taken inside the tile loop.
//
// Every global round trip is kept off a wave's critical path (see
// qhuff_pipeline.h): tiles come from in-order tickets claimed two
// iterations ahead (Tickets), offsets are loaded two tiles ahead and input
// one tile ahead, and a tile's look-back and stores are deferred until
// after the next tile's codec -- its output waits in registers -- so polls
// find their predecessors published and no wait drains freshly issued
// stores.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qhuff {

#define QH_LDS __attribute__((address_space(3)))
#define QH_GLB __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// byte-aligned views for unaligned global stores (gfx9 unaligned mode)
struct __attribute__((packed, aligned(1))) U4 { u32x4 v; };
struct __attribute__((packed, aligned(1))) U1 { uint32_t v; };
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWT = 64;                     // strings per wave tile
#ifndef QH_WAVES
#define QH_WAVES 12
#endif
constexpr int kWaves = QH_WAVES;            // waves per workgroup (per kernel TU)

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
// accumulators kAccStride u64 apart (256 B, a line each): device-scope
// atomics to one line are serialised (~88/us, MI355X_MICROARCH.md
// 'dequeue'), and with 16 accumulators per line every running super tile's
// adds queued on a handful of lines -- the returned add then cost ~3.5k
// cycles of each tile's poll wait (profiles/r02_c/phases_*.txt)
constexpr uint32_t kAccStride = 32;
// tile flags kFlagStride u64 apart (1: dense, a poll window is 4 lines;
// 4 and 16 were equal / 3 % slower, profiles/r02_h/ab_tile_flag_stride.txt)
constexpr uint32_t kFlagStride = 1;

// error bits reported through Coord::err
constexpr uint32_t kErrSpin = 1;            // look-back spin limit hit
constexpr uint32_t kErrRange = 2;           // output offsets passed 2^32

// Dynamic tile tickets: tiles are claimed in order from kTickGroups counters
// (one returning atomic per tile; a single counter saturates near 90
// claims/us on MI355X, MI355X_MICROARCH.md 'dequeue').  Group g (blocks with
// blockIdx % G == g) claims tiles g, g + G, g + 2G, ... in order, so every
// tile a look-back waits on is held by a wave that is running: no
// co-residency assumption.  (12 groups, one per wave of a workgroup, was
// 4 % slower: profiles/r02_r/ab_tick_groups12.txt)
constexpr uint32_t kTickGroups = 8;
// each counter on its own 256-byte span (u32 stride): atomics to one line
// serialise in one L2 channel, and every other access of that channel waits
constexpr uint32_t kTickStride = 64;

struct Coord
{
    unsigned long long *prof;               // QHUFF_PROFILE builds: stamps
    unsigned long long *flags;              // per-tile look-back flags
    unsigned long long *sflags;             // per-super-tile flags
    unsigned long long *sacc;               // super accumulators [2][cap_super],
                                            // kAccStride apart
    uint32_t *tick;                         // tile tickets [2][kTickGroups],
                                            // kTickStride apart
    uint32_t *err;                          // sticky device error word
    uint32_t *err_host;                     // its pinned host mirror
    uint32_t epoch;                         // launch tag carried in flags
    uint32_t n_tiles;
    uint32_t cap_super;                     // sacc entries per parity
    uint32_t spread;                        // > 0: the first `spread` waves of
                                            // each workgroup take one tile
                                            // each from counter 0 (batches
                                            // the grid covers; qhuff_pipeline.h)
    uint8_t *big;                           // big-tile output slots:
                                            // kBigSlots per wave of the grid
};

// A big tile's output (qhuff_pipeline.h) waits in one of its wave's
// kBigSlots global slots of kBigSlotBytes until the tile is flushed: as
// many slots as pending tiles + 1 (the tile coded in an iteration is placed
// before that iteration's flush frees the oldest).
constexpr uint32_t kBigSlots = 4;
constexpr uint32_t kBigSlotBytes = 12288;
constexpr uint32_t kBigMaxWaves = 16;       // per workgroup (host allocation)
static_assert(kWaves <= (int) kBigMaxWaves, "big-tile slots per workgroup");

struct Coord;
__device__ __forceinline__ void raise_error(const Coord &c, uint32_t bits);

// The lane id is opaque to the optimiser (round 6): a per-lane address
// computed from it (a big-tile slot, a 16-byte chunk of a copy) is then
// rebuilt where it is used, not computed once before the tile loop and
// kept -- spilled -- across it.  Full encode 18 -> 2 spilled VGPRs, full
// decode 11 -> 2 (profiles/r06_f).
#ifndef QH_OPAQUE_LANE
#define QH_OPAQUE_LANE 1
#endif
__device__ __forceinline__ uint32_t
lane_id()
{
#if QH_OPAQUE_LANE
    uint32_t v = threadIdx.x & 63;
    asm volatile("" : "+v"(v));
    return v;
#else
    return threadIdx.x & 63;
#endif
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
read_lane(uint32_t v, uint32_t lane)
{
    return __builtin_amdgcn_readlane(v, lane);
}

__device__ __forceinline__ uint64_t
read_lane64(uint64_t v, uint32_t lane)
{
    return ((uint64_t) read_lane((uint32_t) (v >> 32), lane) << 32)
         | read_lane((uint32_t) v, lane);
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

// DPP move of v (gfx9 dpp_ctrl CTRL on rows ROWS); lanes whose source lies
// outside the pattern, or whose row is masked off, read 0
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t
dpp0(uint32_t v)
{
    return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, CTRL, ROWS, 0xf,
                                                  false);
}

// wave inclusive scan of one uint32 per lane: scans of the four 16-lane rows
// by row shifts, then the row totals broadcast down (row_bcast:15 / 31) --
// VALU only, no LDS traffic
__device__ __forceinline__ uint32_t
wave_incl_scan(uint32_t v)
{
    uint32_t x = v;
    x += dpp0<0x111, 0xf>(x);                 // row_shr:1
    x += dpp0<0x112, 0xf>(x);                 // row_shr:2
    x += dpp0<0x114, 0xf>(x);                 // row_shr:4
    x += dpp0<0x118, 0xf>(x);                 // row_shr:8
    x += dpp0<0x142, 0xa>(x);                 // row_bcast:15 -> rows 1, 3
    x += dpp0<0x143, 0xc>(x);                 // row_bcast:31 -> rows 2, 3
    return x;
}

// whole-wave DPP moves (gfx9 wavefront shifts): lane i gets lane i - 1's
// value; lane 0 gets lane 63's (ror) or 0 (shr)
__device__ __forceinline__ uint32_t
wave_ror1(uint32_t v)
{
    return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x13c, 0xf, 0xf,
                                                  false);
}

__device__ __forceinline__ uint32_t
wave_shr1(uint32_t v)
{
    return (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x138, 0xf, 0xf,
                                                  false);
}

// wave maximum by DPP (row shifts, then the row maxima broadcast down), in
// every lane; VALU only
__device__ __forceinline__ uint32_t
wave_max_dpp(uint32_t v)
{
    uint32_t x = v;
    x = max(x, dpp0<0x111, 0xf>(x));          // row_shr:1
    x = max(x, dpp0<0x112, 0xf>(x));          // row_shr:2
    x = max(x, dpp0<0x114, 0xf>(x));          // row_shr:4
    x = max(x, dpp0<0x118, 0xf>(x));          // row_shr:8
    x = max(x, dpp0<0x142, 0xa>(x));          // row_bcast:15 -> rows 1, 3
    x = max(x, dpp0<0x143, 0xc>(x));          // row_bcast:31 -> rows 2, 3
    return read_lane(x, 63);
}

// sum over the wave of values below 2^40 (look-back flag values): two
// 32-bit DPP scans of the low 16 and the high 24 bits, no LDS traffic
__device__ __forceinline__ uint64_t
wave_sum40(uint64_t v)
{
    const uint32_t lo = read_lane(wave_incl_scan((uint32_t) v & 0xffffu), 63);
    const uint32_t hi = read_lane(wave_incl_scan((uint32_t) (v >> 16)), 63);
    return ((uint64_t) hi << 16) + lo;
}

__device__ __forceinline__ uint32_t
wave_max(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        v = max(v, (uint32_t) __shfl_xor((int) v, d, 64));
    return v;
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

// sets error bits in the sticky device word and in its pinned host mirror
// (read by the host at the next batch call, qhuff_host.cpp prepare_launch)
__device__ __forceinline__ void
raise_error(const Coord &c, uint32_t bits)
{
    atomicOr(c.err, bits);
    __hip_atomic_fetch_or(c.err_host, bits, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_SYSTEM);
}

// clears the super accumulators of the next launch on the stream (they use
// the other parity; every thread of the grid helps; all of them, since the
// next launch may hold more tiles than this one)
__device__ __forceinline__ void
clear_next_launch(const Coord &c)
{
    const uint32_t par = (c.epoch + 1) & 1;
    // (the workgroup size as the constant it is: blockDim.x is a vector
    // load from the dispatch packet, and its wait drained every load and
    // atomic of the prologue)
    constexpr uint32_t kBT = 64u * kWaves;
    for (uint32_t i = blockIdx.x * kBT + threadIdx.x; i < c.cap_super;
         i += gridDim.x * kBT)
        __hip_atomic_store(&c.sacc[((uint64_t) par * c.cap_super + i) * kAccStride], 0ull,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x < kTickGroups)
        __hip_atomic_store(&c.tick[(par * kTickGroups + threadIdx.x) * kTickStride],
                           0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tile tickets.  Every wave belongs to one of kTickGroups ticket groups,
// g = (blockIdx.x * kWaves + wave) % kTickGroups, so that the waves of ANY
// single workgroup cover every group: tile k * kTickGroups + g is the k-th
// ticket of group g, tickets of a group are handed out in order, and a
// claimed tile is always held by a running wave.  A look-back only waits on
// tiles with smaller indices, so whatever subset of the grid is resident
// (another kernel, context or process on the GPU), the smallest unfinished
// tile is held by a running wave or claimable by one.  (Groups tied to
// workgroups, e.g. blockIdx % 8, follow the XCD the workgroup runs on: two
// kernels that each miss one XCD could then wait on each other for ever.)
// claim() issues the returning atomic (lane 0) and does not wait for it;
// tile_of() reads the result (after a vmcnt wait).
static_assert(kWaves >= (int) kTickGroups, "a workgroup must cover every ticket group");

struct Tickets
{
    uint32_t g;                             // this wave's group

    __device__ __forceinline__ void init()
    {
        g = (blockIdx.x * (uint32_t) kWaves + (threadIdx.x >> 6)) % kTickGroups;
    }
    __device__ __forceinline__ uint32_t *counter(const Coord &c, uint32_t q) const
    {
        return &c.tick[((c.epoch & 1) * kTickGroups + q) * kTickStride];
    }
    // claims `m` consecutive tickets of the group; returns the first
    __device__ __forceinline__ uint32_t claim(const Coord &c, uint32_t m = 1) const
    {
        uint32_t k = 0, q = g;
        // (the opaque copy keeps the counter address from being hoisted
        // out of the tile loop: held there it was a spilled register pair)
        asm volatile("" : "+v"(q));
        if (lane_id() == 0)
            k = __hip_atomic_fetch_add(counter(c, q), m, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        return k;
    }
    // tile of ticket k (wave-uniform; ~0u past 2^32 tiles)
    __device__ __forceinline__ uint32_t tile_of_u(uint32_t k) const
    {
        const uint64_t t = (uint64_t) k * kTickGroups + g;
        return t < 0xffffffffull ? (uint32_t) t : 0xffffffffu;
    }
    // tile of a ticket claim()ed by lane 0
    __device__ __forceinline__ uint32_t tile_of(uint32_t k) const
    {
        return tile_of_u(read_lane(k, 0));
    }
};

// ---- profile stamps (QHUFF_PROFILE builds only) --------------------------
// Stamp slot `ph` of iteration `it` of this wave: prof[(gid * kProfIters +
// it) * kProfSlots + ph] = s_memtime.  Compiled out otherwise.
constexpr int kProfIters = 16, kProfSlots = 12;
__device__ __forceinline__ void
prof_value(const Coord &c, uint32_t it, int ph, uint64_t v)
{
#ifdef QHUFF_PROFILE
    if (c.prof && it < (uint32_t) kProfIters && (threadIdx.x & 63) == 0)
    {
        const uint64_t gid = blockIdx.x * (uint64_t) kWaves + (threadIdx.x >> 6);
        c.prof[(gid * kProfIters + it) * kProfSlots + ph] = v;
    }
#else
    (void) c;
    (void) it;
    (void) ph;
    (void) v;
#endif
}

// s_memrealtime (100 MHz) into slot ph: with s_memtime stamps it gives the
// shader clock the kernel ran at (MI355X_MICROARCH.md, DVFS item 6)
__device__ __forceinline__ void
prof_realtime(const Coord &c, uint32_t it, int ph)
{
#ifdef QHUFF_PROFILE
    prof_value(c, it, ph, __builtin_amdgcn_s_memrealtime());
#else
    (void) c;
    (void) it;
    (void) ph;
#endif
}

__device__ __forceinline__ void
prof_stamp(const Coord &c, uint32_t it, int ph)
{
#ifdef QHUFF_PROFILE
    prof_value(c, it, ph, __builtin_amdgcn_s_memtime());
#else
    (void) c;
    (void) it;
    (void) ph;
#endif
}

// ---- tile offsets ------------------------------------------------------

// Lane i holds the start offset of string i of the tile and of string i+1
// (clamped to the tile end).  `cnt` strings, cnt in [1, 64].  Both loads are
// issued by every lane (clamped index): a fixed instruction count keeps the
// compiler's vmcnt waits exact.
struct TileOffs
{
    uint32_t o0, o1;

    __device__ __forceinline__ void load(const QH_GLB uint32_t *in_off,
                                         uint64_t s0, uint32_t cnt)
    {
        const uint32_t lane = lane_id();
        o0 = in_off[s0 + (lane < cnt ? lane : cnt)];
        // (o1 as the next lane's o0 by a DPP shift + one uniform load was
        // slower: enc 64.8 vs 63.4, dec 67.9 vs 66.7 us, r02_o/ab_off1.txt)
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
    uint32_t staged;                 // (wave-uniform; see Pending::valid)
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
// write: NCH 16-byte chunks per lane.  Every lane issues every load (index
// clamped into the span), so the instruction count is fixed.
template <int NCH>
struct Chunks
{
    u32x4 ch[NCH];

    __device__ __forceinline__ void load(const Span &sp)
    {
        const uint32_t lane = lane_id();
        const uint32_t last = sp.n16 ? sp.n16 - 1 : 0;
#pragma unroll
        for (int k = 0; k < NCH; ++k)
        {
            const uint32_t i = lane + 64u * k;
            ch[k] = ((const QH_GLB u32x4 *) sp.pa)[i < last ? i : last];
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
// the super tile's aggregate (at the top of its wave's next iteration, when
// the add has long returned).  A tile's exclusive prefix is then
//   (aggregates of the earlier tiles of its super tile, back to an
//    inclusive one if there is one)
// + (super aggregates back to an inclusive super flag),
// one 64-wide window of each, polled together.  Only aggregates are waited
// for, so no wait chains through other look-backs.  The last tile of a super
// tile publishes the super tile's inclusive flag.

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

// s_sleep between look-back polls after the fourth (x 64 cycles): waits
// that long are for a slow tile (the drain at a batch's end), where the
// polls of ~3,000 waves compete with the last codecs' own traffic (with the
// re-polls of invalid flags only: encode -1.5 ... -1.8 %, decode -0.1 ...
// -1.2 %, profiles/r04_y)
#ifndef QH_SPIN_BACKOFF
#define QH_SPIN_BACKOFF 8
#endif

struct LookBack
{
    uint32_t tile, s;
    uint32_t total;
    uint64_t acc_old;            // returned by the super accumulator add (lane 0)
    uint64_t ft, fs, fs1;        // polled tile flags, super flags back 0 / 1
#ifdef QHUFF_PROFILE
    uint32_t spins_seen;         // re-polls of the last finish() (profiling)
#endif

    __device__ __forceinline__ static uint64_t ep(const Coord &c)
    {
        return (uint64_t) c.epoch << 42;
    }
    __device__ __forceinline__ uint64_t poll_tile(const Coord &c) const
    {
        const uint32_t lane = lane_id();
        const uint32_t nq = tile - s * kSuper;
        // lanes past the super start re-read the nearest valid slot
        const uint32_t q = lane < nq ? lane : (nq ? nq - 1 : 0);
        // (the raw flag: finish() masks lanes past nq; no use of the loaded
        // value here, so the poll's latency is not waited for until then)
        return __hip_atomic_load(&c.flags[(uint64_t) (nq ? tile - 1 - q : tile) * kFlagStride],
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // super flags s-1-lane-64*back, raw (see super_val)
    __device__ __forceinline__ uint64_t poll_super(const Coord &c,
                                                   uint32_t back) const
    {
        const int64_t j = (int64_t) s - 1 - lane_id() - 64 * (int64_t) back;
        return __hip_atomic_load(&c.sflags[j < 0 ? 0 : j], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    }
    // a polled super flag; before super 0: inclusive 0
    __device__ __forceinline__ uint64_t super_val(const Coord &c, uint32_t back,
                                                  uint64_t f) const
    {
        const int64_t j = (int64_t) s - 1 - lane_id() - 64 * (int64_t) back;
        return j < 0 ? (kFlagInc | ep(c)) : f;
    }

    // the look-back of tile t (total tot) whose aggregate is published
    __device__ __forceinline__ void at(uint32_t t, uint32_t tot)
    {
        tile = t;
        s = t / kSuper;
        total = tot;
    }
    // publish the aggregate, add to the super accumulator
    __device__ __forceinline__ void start(const Coord &c, uint32_t t,
                                          uint32_t tot)
    {
        tile = t;
        s = t / kSuper;
        total = tot;
        acc_old = 0;
        if (lane_id() == 0)
        {
            __hip_atomic_store(&c.flags[(uint64_t) t * kFlagStride], kFlagAgg | ep(c) | tot,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc_old = __hip_atomic_fetch_add(
                &c.sacc[((uint64_t) (c.epoch & 1) * c.cap_super + s) * kAccStride],
                kAccOne + tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __device__ __forceinline__ void publish_super(const Coord &c, uint64_t state,
                                                  uint64_t v) const
    {
        if (lane_id() == 0)
            __hip_atomic_fetch_max(&c.sflags[s], state | ep(c) | (v & kValMask),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the add that completed the super tile publishes its aggregate
    __device__ __forceinline__ void super_agg(const Coord &c) const
    {
        const uint32_t f0 = s * kSuper;
        const uint32_t in_super = c.n_tiles - f0 < (uint32_t) kSuper
                                ? c.n_tiles - f0 : (uint32_t) kSuper;
        const uint64_t old = read_lane64(acc_old, 0);
        if ((old >> 48) == in_super - 1)
            publish_super(c, kFlagAgg, (old + total) & kAccMask);
    }
    // the tile window and two super windows (128 super tiles): with ~2
    // iterations of ~3,000-4,000 waves between a tile's codec and its
    // inclusive flag, the nearest inclusive super flag is 100-130 super tiles
    // back, so one window would cost a second round trip on most tiles
    __device__ __forceinline__ void poll(const Coord &c)
    {
        ft = poll_tile(c);
        fs = poll_super(c, 0);
        fs1 = poll_super(c, 1);
    }

    __device__ __forceinline__ bool spin(const Coord &c, uint32_t *spins) const
    {
        if (++*spins > kSpinLimit)
        {
            if (lane_id() == 0)
                raise_error(c, kErrSpin);
            return false;
        }
#if QH_SPIN_BACKOFF
        if (*spins > 4)
            __builtin_amdgcn_s_sleep(QH_SPIN_BACKOFF);
        else
#endif
        __builtin_amdgcn_s_sleep(2);
        return true;
    }

    // returns the exclusive prefix of the tile (polls issued by poll());
    // publishes its inclusive one
    __device__ __forceinline__ uint64_t finish(const Coord &c)
    {
        const uint32_t lane = lane_id();
        const uint32_t f0 = s * kSuper;
        const uint32_t nq = tile - f0;               // earlier tiles in super
        uint32_t spins = 0;
        uint64_t excl = 0;
        // 1. earlier tiles of this super tile
        bool done = false;
        for (;;)
        {
            const bool inq = lane < nq;
            const bool v = flag_valid(ft, c.epoch);
            const uint64_t inv = __ballot(inq && !v);
            const uint64_t inc = __ballot(inq && v && flag_inc(ft));
            const int F = inc ? __builtin_ctzll(inc) : 64;
            const uint64_t upto = F >= 63 ? ~0ull : ((2ull << F) - 1);
            if ((inv & upto) == 0)
            {
                excl = wave_sum40((inq && (int) lane <= F) ? (ft & kValMask)
                                                           : 0ull);
                done = inc != 0;
                break;
            }
            if (!spin(c, &spins))
            {
                done = true;
                break;
            }
            // re-poll only the flags not yet valid: an aggregate is final
            // (a valid flag turning inclusive only shortens the sum), and a
            // wave waiting for a slow tile -- every wave in the drain at the
            // end of a batch -- then reads one or two cache lines a poll,
            // not the window's eight
            if (!v)
                ft = poll_tile(c);
        }
        const uint32_t spins1 = spins;
        uint32_t extra = 0;                          // windows past the two
        // 2. super tiles before this one, back to an inclusive one
        for (uint32_t back = 0; !done;)
        {
            const uint64_t fv = super_val(c, back, fs);
            const bool v = flag_valid(fv, c.epoch);
            const uint64_t inv = __ballot(!v);
            const uint64_t inc = __ballot(v && flag_inc(fv));
            const int G = inc ? __builtin_ctzll(inc) : 64;
            const uint64_t upto = G >= 63 ? ~0ull : ((2ull << G) - 1);
            if ((inv & upto) == 0)
            {
                excl += wave_sum40((int) lane <= G ? (fv & kValMask) : 0ull);
                if (inc)
                    break;
                ++back;
                // the second window was polled with the first
                fs = back == 1 ? fs1 : poll_super(c, back);
                extra += back > 1 ? 1u : 0u;
                continue;
            }
            if (!spin(c, &spins))
                break;
            if (!v)                                  // (as above)
                fs = poll_super(c, back);
        }
        // Every poll has been consumed, so nothing is outstanding here but
        // the compiler cannot see that the re-poll loads (whose registers the
        // flush reuses) have landed: without this wait it puts a vmcnt(0)
        // into each partial-chunk store path of the flush, where it drains
        // the tile's own dwordx4 stores issued just before (~2k cycles).
        __builtin_amdgcn_s_waitcnt(0x0f70);
        if (lane == 0)
            __hip_atomic_store(&c.flags[(uint64_t) tile * kFlagStride],
                               kFlagInc | ep(c) | ((excl + total) & kValMask),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t in_super = c.n_tiles - f0 < (uint32_t) kSuper
                                ? c.n_tiles - f0 : (uint32_t) kSuper;
        if (tile == f0 + in_super - 1)
            publish_super(c, kFlagInc, excl + total);
#ifdef QHUFF_PROFILE
        spins_seen = spins1 | ((spins - spins1) << 12) | (extra << 24);
#else
        (void) spins1;
        (void) extra;
#endif
        return excl;
    }
};

// ---- deferred output --------------------------------------------------------

// A tile's compacted output (at most 64 * NCH * 16 bytes) held in registers
// between its gather from the LDS stage and its store: lane l holds the
// tile-local 16-byte chunks l, l + 64, ...  store() shifts them to the
// alignment of the global destination with one cross-lane rotate per dword,
// writes whole 16-byte chunks with dwordx4 stores and the partial first / last
// chunk with one byte store (lanes 0-15 and 16-31), so a tile's stores are a
// fixed number of instructions.
template <int NCH>
struct TileOut
{
    u32x4 o[NCH];

    __device__ __forceinline__ void clear()
    {
#pragma unroll
        for (int j = 0; j < NCH; ++j)
            o[j] = (u32x4){0, 0, 0, 0};
    }
    __device__ __forceinline__ void gather(const QH_LDS uint32_t *stage)
    {
        const uint32_t lane = lane_id();
#pragma unroll
        for (int j = 0; j < NCH; ++j)
            o[j] = ((const QH_LDS u32x4 *) stage)[lane + 64 * j];
    }

    // Global stores of the tile's `total` bytes at dst (any alignment: the
    // ROCm driver runs gfx9 in unaligned-access mode, and the 16-byte stores
    // of neighbouring lanes and tiles never overlap).  Whole 16-byte chunks:
    // one dwordx4 store per lane; the partial last chunk: its owner lane
    // writes its whole dwords, then its last 0-3 bytes.
    __device__ __forceinline__ void store(uint8_t *dst, uint32_t total) const
    {
        const uint32_t lane = lane_id();
        const uint32_t nfull = total >> 4, rem = total & 15;
        // the lane's byte offset comes out of an opaque instruction here, at
        // the store: left to itself the compiler hoists the 64-bit per-lane
        // offset out of the tile loop and, at depth 3, spills it (a scratch
        // reload and a vmcnt(0) before every flush)
        uint32_t lo;
        asm volatile("v_lshlrev_b32 %0, 4, %1" : "=v"(lo) : "v"(lane));
        // (compile-time chunk index j throughout: a run-time select between
        // the o[] would put the array in scratch memory)
#pragma unroll
        for (int j = 0; j < NCH; ++j)
        {
            const uint32_t k = lane + 64u * j;
            uint8_t *p = dst + (lo + 1024u * j);
            if (k < nfull)
                ((QH_GLB U4 *) p)->v = o[j];
            else if (k == nfull && rem)
                store_part(p, o[j], rem);
        }
    }
    __device__ __forceinline__ static void store_part(uint8_t *dst, u32x4 v,
                                                      uint32_t rem)
    {
        QH_GLB uint8_t *p = (QH_GLB uint8_t *) dst;
        const uint32_t nd = rem >> 2;
        if (nd > 0)
            ((QH_GLB U1 *) p)->v = v.x;
        if (nd > 1)
            ((QH_GLB U1 *) (p + 4))->v = v.y;
        if (nd > 2)
            ((QH_GLB U1 *) (p + 8))->v = v.z;
        const uint32_t wt = nd == 0 ? v.x : nd == 1 ? v.y : nd == 2 ? v.z : v.w;
        const uint32_t nb = rem & 3;
        QH_GLB uint8_t *q = p + 4 * nd;
        if (nb > 0)
            q[0] = (uint8_t) wt;
        if (nb > 1)
            q[1] = (uint8_t) (wt >> 8);
        if (nb > 2)
            q[2] = (uint8_t) (wt >> 16);
    }
};

}  // namespace qhuff
