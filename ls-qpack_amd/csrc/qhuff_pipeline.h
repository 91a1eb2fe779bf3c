// qhuff_pipeline.h -- the per-wave tile loop shared by the encode and decode
// kernels (see qhuff_device.h for the execution model).
//
// Tiles come from in-order tickets (qhuff_device.h Tickets): a wave's
// first two tiles from one claim per block in the kernel prologue, then one
// claim per iteration for the tile two iterations ahead -- every tile a
// look-back waits on belongs to a running wave, whatever the residency.
// Per iteration, for tile t:
//
//   top    one wait for what the last iteration issued: t's input chunks (a
//          codec ago), the next tile's offsets, the stores of the last
//          iteration.  P::stage_in()
//          -- t's chunks into the LDS stage -- then the loads of the next
//          tile's input, the claim of the tile after it, and the older
//          pending tile's look-back polls: all of them have the whole codec
//          to land
//   codec  P::prepare() (the encoder's byte-parallel pass over the stage),
//          P::codec() -- LDS only -- per-lane output size (+ status)
//   scan   wave scan -> tile-local offsets, tile total; publish the tile
//          aggregate and add it to the super accumulator (LookBack::start)
//   emit   P::emit() -- compacted output of t into the LDS out stage
//   flush  one wait (the polls and the claim, a codec and an emit ago, and
//          t's super add); the claimed tile's offsets loads; publish t's
//          super tile's aggregate if t's add completed it; resolve the older
//          pending tile's look-back and store its output (registers)
//   gather t's output from the out stage into the freed registers (TileOut)
//
// P::kDepth tiles are pending at a time, all holding their output in
// registers: tile k's look-back windows are polled at the top of iteration
// k + kDepth, kDepth - 1 whole iterations after every tile before it
// published its aggregate, and resolved after that iteration's codec and
// emit.  (A wave held up in a look-back delays its own next codecs, and so
// the look-backs of the tiles after those: the deeper the pipeline, the more
// slack before such a delay propagates.)
//
// Tiles whose input or output does not fit the stages are big tiles: coded
// in staged units into a global slot and pending like any other (full
// kernels, P::kBig), or by P::slow_tile() out of line after the pending
// tiles have been flushed (lean kernels, and a big tile past its slot).
#pragma once

#include "qhuff_kernels.h"


namespace qhuff {

// youngest waves' claims stop QH_TAIL_STOP quarter-rounds before the end
// (tile_pipeline; 6: -0.6 % on average over four same-box pairs, 2 and 4
// neutral, 8 and 12 +3 ... +6 %: profiles/r04_z, r04_z2)
#ifndef QH_TAIL_STOP
#define QH_TAIL_STOP 6
#endif

// a rare branch of the full kernels' tile loop (their cooperative phase,
// big tiles): marked cold there, so that block and spill placement favour
// the loop (full kernels on the token batch: encode 0.955, decode 0.982,
// profiles/r05_cold); the lean kernels' loop is left as it was (the same
// hints cost their decode ~1 %)
#define QH_RARE(full, c) ((full) ? __builtin_expect((c), 0) : (c))
#ifndef QH_COOP_VIA_BIG
#define QH_COOP_VIA_BIG 1
#endif

constexpr int kChunks = 3;                  // 16-byte input chunks per lane
constexpr int kStageCap = 64 * kChunks * 16;  // 3072 B: chunk registers / stages

// A coded tile waiting for its look-back: per-lane output offset and status,
// its tile and total; its output bytes wait in registers (TileOut).  (The
// look-back state -- polls -- lives only for the tile being resolved: kept
// per pending tile it cost ~14 VGPRs a tile.)
struct Pending
{
    uint32_t valid;                  // (wave-uniform; a bool here is a lane mask)
    uint32_t excl;                   // this lane's tile-local output offset
    uint32_t stat;                   // this lane's status byte
    uint32_t tile, total;            // (wave-uniform)
    uint32_t big;                    // (wave-uniform) a big tile: 1 + its
                                     // output slot; 0: output in TileOut
    __device__ __forceinline__ LookBack lb() const
    {
        LookBack l;
        l.at(tile, total);
        return l;
    }
};

// A cross-lane result (DPP, ds_bpermute), computed by every lane here: left
// to itself the compiler may move the operation into the branch of a select
// that uses it, where the lanes it reads from are off (and read as 0).
template <class T>
__device__ __forceinline__ T
all_lanes(T v)
{
    asm volatile("" : "+v"(v));
    return v;
}

// Output base of a slow tile (P::slow_tile / slow_tile_at): the batch
// kernel's look-back, or a base the caller already has (the service kernel
// codes a request's tiles in order in one wave).
struct LookBackBase
{
    Coord c;
    uint32_t t;
    __device__ __forceinline__ uint64_t operator()(uint32_t total) const
    {
        LookBack lb;
        lb.start(c, t, total);
        lb.super_agg(c);
        lb.poll(c);
        return lb.finish(c);
    }
};
// ... or a look-back already started (its aggregate published, its super
// add returned: the batch kernel's slow tiles, published before the wave's
// pending tiles are flushed)
struct StartedBase
{
    Coord c;
    LookBack lb;
    __device__ __forceinline__ uint64_t operator()(uint32_t)
    {
        lb.poll(c);
        return lb.finish(c);
    }
};
struct FixedBase
{
    uint64_t base;
    __device__ __forceinline__ uint64_t operator()(uint32_t) const
    {
        return base;
    }
};

// the batch's last tile: the closing offset (and the 32-bit range check)
__device__ __forceinline__ void
last_tile_end(const Coord &c, uint32_t t, uint64_t end, uint32_t *out_off,
              uint64_t n)
{
    if (t == c.n_tiles - 1 && lane_id() == 0)
    {
        ((QH_GLB uint32_t *) out_off)[n] = (uint32_t) end;
        if (end > 0xffffffffull)                 // offsets are 32-bit
            raise_error(c, kErrRange);
    }
}

// (big tiles, qhuff_*_impl.h) the tile's lanes [i0, i0 + k) whose 16-byte-aligned input span fits the
// stage (and, with outputs, whose output leaves 64 bytes of it free): k
// (offsets ascend, so they are a prefix of the lanes from i0)
__device__ __forceinline__ uint32_t
unit_len(const uint8_t *in, const TileOffs &to, uint32_t i0, uint32_t cnt,
         uint32_t cap, bool outs, uint32_t excl, uint32_t sz, uint32_t ocap)
{
    const uint32_t lane = lane_id();
    const uintptr_t pa = (uintptr_t) (in + read_lane(to.o0, i0)) & ~(uintptr_t) 15;
    const uintptr_t pe = ((uintptr_t) (in + to.o1) + 15) & ~(uintptr_t) 15;
    const uint32_t e0 = read_lane(excl, i0);
    const bool fit = (lane >= i0) & (lane < cnt) & (pe - pa <= (uintptr_t) cap)
                   & (!outs | (excl + sz - e0 + 64 <= ocap));
    return (uint32_t) __builtin_popcountll(__builtin_amdgcn_ballot_w64(fit));
}

// n bytes of LDS at src -> global dst (any alignment), the whole wave:
// 16-byte stores (unaligned-access mode, as TileOut::store), the last < 16
// bytes one per lane
__device__ __forceinline__ void
copy_out(const QH_LDS uint8_t *src, uint8_t *dst, uint32_t n)
{
    const uint32_t lane = lane_id();
    const uint32_t sa = (uint32_t) (uintptr_t) src, r = sa & 3;
    const QH_LDS uint32_t *sw = (const QH_LDS uint32_t *) (src - r);
    const uint32_t n16 = n >> 4;
    for (uint32_t i = lane; i < n16; i += 64)
    {
        const QH_LDS uint32_t *w = sw + 4 * i;
        const uint32_t a = w[0], b = w[1], c = w[2], d = w[3], e = w[4];
        ((QH_GLB U4 *) (dst + 16 * i))->v =
            (u32x4){align_bytes(b, a, r), align_bytes(c, b, r),
                    align_bytes(d, c, r), align_bytes(e, d, r)};
    }
    const uint32_t t = 16 * n16 + lane;
    if (lane < 16 && t < n)
        ((QH_GLB uint8_t *) dst)[t] = src[t];
}

// a span's (<= 3 KB) 16-byte chunks global -> LDS (big tiles,
// qhuff_*_impl.h): the lane's three loads issued together, then stored
template <bool SWAP>
__device__ __forceinline__ void
stage_chunks(const Span &sp, QH_LDS u32x4 *dst)
{
    const uint32_t l = lane_id();
    const uint32_t last = sp.n16 ? sp.n16 - 1 : 0;
    const QH_GLB u32x4 *src = (const QH_GLB u32x4 *) sp.pa;
    u32x4 v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        v[k] = src[min(l + 64u * k, last)];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (l + 64u * k < sp.n16)
        {
            u32x4 x = v[k];
            if (SWAP)
                x = (u32x4){bswap32(x.x), bswap32(x.y), bswap32(x.z),
                            bswap32(x.w)};
            dst[l + 64u * k] = x;
        }
    wave_sync();
}

// this wave's big-tile output slot k (Coord::big)
__device__ __forceinline__ uint8_t *
big_slot(const Coord &c, uint32_t k)
{
    // (wave-uniform, scalar: in a VGPR pair this address was computed
    // before the tile loop and spilled across it)
    const uint64_t gid = (uint64_t) blockIdx.x * kWaves
                       + (uint32_t) __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return c.big + (gid * kBigSlots + k) * (uint64_t) kBigSlotBytes;
}

// n bytes of a big-tile slot -> dst (any alignment), the whole wave.  The
// slot was written by this wave a few iterations ago and is read back
// through L2 (agent-scope loads): an earlier read of the same slot may
// still sit in this CU's L1.
__device__ __forceinline__ void
copy_slot(const uint8_t *src, uint8_t *dst, uint32_t n)
{
    const uint32_t lane = lane_id();
    const QH_GLB uint32_t *s = (const QH_GLB uint32_t *) src;
    auto ld = [&](uint32_t w) -> uint32_t {
        return __hip_atomic_load(s + w, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    };
    const uint32_t n16 = n >> 4;
    for (uint32_t i = lane; i < n16; i += 64)
        ((QH_GLB U4 *) (dst + 16 * i))->v =
            (u32x4){ld(4 * i), ld(4 * i + 1), ld(4 * i + 2), ld(4 * i + 3)};
    const uint32_t t = 16 * n16 + lane;
    if (lane < 16 && t < n)
        ((QH_GLB uint8_t *) dst)[t] = (uint8_t) (ld(t >> 2) >> (8 * (t & 3)));
}

// resolve a pending tile's base and store it from `o` (every lane)
template <class P>
__device__ __forceinline__ void
flush_tile(const Coord &c, Pending &d, LookBack &lb, const TileOut<P::kNch> &o,
           uint8_t *out, uint32_t *out_off, uint8_t *status, uint64_t n,
           uint32_t it = ~0u)
{
    const uint64_t base = lb.finish(c);
    prof_stamp(c, it, 7);
#ifdef QHUFF_PROFILE
    prof_value(c, it, 8, lb.spins_seen);
#endif
    // (wave-uniform: readfirstlane lets the offsets / status addresses
    // live in SGPRs)
    const uint32_t tile = __builtin_amdgcn_readfirstlane(d.tile);
    const uint32_t total = d.total;
    if (__builtin_expect(d.big != 0, 0))
        copy_slot(big_slot(c, d.big - 1), out + base, total);
    else
        o.store(out + base, total);
    uint32_t lane = lane_id();
    // (opaque: the per-lane addresses are rebuilt here, not hoisted out of
    // the tile loop as a register pair each)
    asm volatile("" : "+v"(lane));
    const uint64_t s0 = (uint64_t) tile * P::kTS;
    const uint32_t cnt = (uint32_t) min((uint64_t) P::kTS, n - s0);
    if (lane < cnt)
    {
        ((QH_GLB uint32_t *) out_off)[s0 + lane] = (uint32_t) (base + d.excl);
        if (P::kStatus)
            ((QH_GLB uint8_t *) status)[s0 + lane] = (uint8_t) d.stat;
    }
    if (tile == c.n_tiles - 1 && lane == 0)
    {
        ((QH_GLB uint32_t *) out_off)[n] = (uint32_t) (base + total);
        if (base + total > 0xffffffffull)        // offsets are 32-bit
            raise_error(c, kErrRange);
    }
    d.valid = false;
}

// vmcnt(0), other counters untouched (gfx9 s_waitcnt encoding)
__device__ __forceinline__ void
wait_vm_all()
{
    __builtin_amdgcn_s_waitcnt(0x0f70);
}

// The kernel prologue claims the first tickets of every wave of the
// workgroup: lanes 0..kTickGroups-1 of the first wave each take one group's
// share with one returning atomic (~3,000 waves claiming one by one would
// queue on the counters).  A wave of group g that is the r-th of its group
// in the workgroup gets tickets base + r, base + n_g + r and base + 2 n_g + r
// (n_g waves of the workgroup in group g).  Two tickets per wave (the
// kernels' maxper; three when maxper allows it and the tiles cover three
// per wave of the whole grid); a ticket not claimed here is kClaimNow: the
// wave claims it itself once it runs, like every later one.
// Every wave goes on claiming until a claim lands past the end, so no
// ticket of any group is left to a workgroup that is not running -- a tile
// fixed to whichever workgroup claimed it would need the whole grid
// resident: with only some workgroups resident, e.g. beside another
// context, a group's tickets could run ahead of another's and the
// look-backs above the gap wait for tiles no running wave can claim.  (The
// one-ticket-per-wave launch of rounds 2-3, where no wave claimed again,
// had exactly that hole; it is gone.)  Batches of at most one tile per wave
// of the grid are spread instead (Coord::spread > 0, qhuff_host.cpp
// grid_for): workgroup b's thread 0 adds `spread` to counter 0 alone and
// its first `spread` waves take those tiles, one each; the claimed tiles
// are always a prefix, so the same holds.
constexpr uint32_t kClaimNow = 0xffffffffu;   // ticket: claim it in the wave
                                              // (tile_pipeline)
struct BlockTickets
{
    uint32_t base[kTickGroups];
    uint32_t per;                    // tickets claimed per wave (1..3)
};

__device__ __forceinline__ uint32_t
tick_group_waves(uint32_t q)
{
    // waves w of this workgroup with (blockIdx.x * kWaves + w) % G == q
    const uint32_t s = (blockIdx.x * (uint32_t) kWaves) % kTickGroups;
    const uint32_t first = (q + kTickGroups - s) % kTickGroups;
    return first < (uint32_t) kWaves
         ? ((uint32_t) kWaves - 1 - first) / kTickGroups + 1 : 0u;
}

// tickets claimed per wave in the prologue (ticket-group launches hold more
// tiles than the grid has waves: smaller batches are spread)
__device__ __forceinline__ uint32_t
block_claims_per_wave(const Coord &c, uint32_t maxper)
{
    const uint64_t g = (uint64_t) gridDim.x * kWaves;
    return (uint64_t) c.n_tiles >= 3 * g && maxper >= 3 ? 3u : 2u;
}

// the atomic of this thread's group share (threads 0..kTickGroups-1; its
// value is waited for only where it is stored: claim_block_store)
__device__ __forceinline__ uint32_t
claim_block_issue(const Coord &c, const Tickets &tk, uint32_t maxper)
{
    const uint32_t t = threadIdx.x;
    uint32_t b = 0;
    if (c.spread)
    {
        // one counter, `spread` consecutive tiles per workgroup
        if (t == 0)
            b = __hip_atomic_fetch_add(tk.counter(c, 0), c.spread,
                                       __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
    else if (t < kTickGroups)
    {
        const uint32_t nq = tick_group_waves(t);
        if (nq)
            b = __hip_atomic_fetch_add(tk.counter(c, t),
                                       block_claims_per_wave(c, maxper) * nq,
                                       __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
    return b;
}

__device__ __forceinline__ void
claim_block_store(const Coord &c, uint32_t b, QH_LDS BlockTickets *bt,
                  uint32_t maxper)
{
    const uint32_t t = threadIdx.x;
    if (t < kTickGroups)
        bt->base[t] = b;
    if (t == 0)
        bt->per = c.spread ? 1u : block_claims_per_wave(c, maxper);
}

__device__ __forceinline__ void
claim_block_tickets(const Coord &c, const Tickets &tk, QH_LDS BlockTickets *bt,
                    uint32_t maxper)
{
    claim_block_store(c, claim_block_issue(c, tk, maxper), bt, maxper);
}

// this wave's first tile t0 and its next tickets (after the workgroup
// barrier)
__device__ __forceinline__ void
wave_tickets(const Coord &c, const Tickets &tk, const QH_LDS BlockTickets *bt,
             uint32_t *t0, uint32_t *k1, uint32_t *k2)
{
    if (c.spread)
    {
        const uint32_t w = threadIdx.x >> 6;
        *t0 = w < c.spread ? bt->base[0] + w : 0xffffffffu;
        *k1 = *k2 = kClaimNow;
        return;
    }
    // rank among this workgroup's waves of the same group (waves w and
    // w + kTickGroups share one)
    const uint32_t r = (threadIdx.x >> 6) / kTickGroups;
    const uint32_t nq = tick_group_waves(tk.g);
    const uint32_t per = bt->per;
    *t0 = tk.tile_of_u(bt->base[tk.g] + r);
    *k1 = per >= 2 ? bt->base[tk.g] + nq + r : kClaimNow;
    *k2 = per >= 3 ? bt->base[tk.g] + 2 * nq + r : kClaimNow;
}

// no work between the first offsets loads and the first wait
struct NoMid
{
    __device__ __forceinline__ void operator()() const {}
};

// mid(): called once by every wave after its first offsets loads have been
// issued, before anything waits for them (the decode kernel stores its
// window table and joins the workgroup barrier there, so the loads overlap
// the table's); every wave of the workgroup calls it, tiles or none.
template <class P, class Mid = NoMid>
__device__ __forceinline__ void
tile_pipeline(P &pol, const Coord &c, const Tickets &tk, uint32_t t0,
              uint32_t k1, uint32_t k2, const uint8_t *in,
              const uint32_t *in_off_p, uint64_t n, uint8_t *out,
              uint32_t *out_off, uint8_t *status, Mid mid = Mid())
{
    const QH_GLB uint32_t *in_off = (const QH_GLB uint32_t *) in_off_p;
    const uint32_t nt = c.n_tiles;
    // this wave's first tile t0 and the tickets k1 < k2 of its next ones
    // (claimed for the whole block in the kernel prologue, or kClaimNow)
    uint32_t t = t0;
    if (t >= nt)
    {
        mid();
        return;
    }
    constexpr uint32_t TS = P::kTS;          // strings per tile
    auto cnt_of = [&](uint32_t tt) -> uint32_t {
        return (uint32_t) min((uint64_t) TS, n - (uint64_t) tt * TS);
    };
    // the loads for tile ids past the end read the last tile instead
    // (fixed instruction counts; the data is never used)
    auto clamp = [&](uint32_t tt) -> uint32_t {
        return tt < nt ? tt : nt - 1;
    };

    // prologue: offsets of t and tn, input of t (landed at the top), the
    // ticket of the third iteration
    typename P::Offs o_cur, o_nxt, o_nn;
    o_cur.load(in_off, (uint64_t) t * TS, cnt_of(t));
    // (a spread launch's wave has one tile and no ticket after it)
    uint32_t tn = k1 == kClaimNow ? 0xffffffffu : tk.tile_of_u(k1);
    o_nxt.load(in_off, (uint64_t) clamp(tn) * TS, cnt_of(clamp(tn)));
    // a wave claims another tile only while its next one is real: a claimed
    // tile is always coded (tickets of a group are handed out in order, so
    // once tn is past the end every later claim is too)
    const uint32_t kNone = 0xffffffffu;
    // the ticket of the third iteration when the workgroup claimed it
    uint32_t kpre = tn < nt ? k2 : kNone;
    // The youngest waves of each SIMD (w >= kTickGroups: the first
    // kTickGroups waves of any workgroup cover every ticket group, so these
    // may stop claiming without leaving a ticket unclaimed) code a tile ~40 %
    // slower than the oldest (profiles/r04_s): they stop claiming once their
    // next tile is within QH_TAIL_STOP quarter-rounds of the grid of the end,
    // so that the batch's last tiles go to faster waves.
    uint32_t stop_fr = 0xffffffffu;          // (wave-uniform)
#if QH_TAIL_STOP
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= (int) kTickGroups)
    {
        const uint32_t q = gridDim.x * (uint32_t) kWaves * QH_TAIL_STOP / 4;
        stop_fr = nt > q ? nt - q : 0u;
    }
#endif
    mid();
    Span sp_cur = tile_span(in, o_cur.first(), o_cur.last(), P::kInCap);
    Chunks<P::kNch> ch;
    ch.load(sp_cur);

    // Tiles come from in-order tickets claimed two iterations ahead (one
    // claim per wave per iteration), so the order in which a wave claims
    // tiles is the order in which it codes them, and a look-back only ever
    // waits on tiles held by running waves.  Between its codec and its
    // store a tile's output sits in registers: P::kDepth pending tiles,
    // oldest first (compile-time indices only: the arrays stay in
    // registers).
    constexpr int D = P::kDepth;
    Pending pend[D];
    TileOut<P::kNch> outs[D];
    // resolve + store pending tile i (compile-time i), polled into lb
    auto flush_at = [&](int i, LookBack &lb, uint32_t itn) {
        flush_tile<P>(c, pend[i], lb, outs[i], out, out_off, status, n, itn);
    };
#pragma unroll
    for (int i = 0; i < D; ++i)
    {
        pend[i].valid = false;
        pend[i].big = 0;
    }
    uint32_t big_next = 0;                   // big-tile slots used (ring)
    uint32_t it = 0;
    for (;; ++it)
    {
        prof_stamp(c, it, 0);
        prof_realtime(c, it, 11);            // 100 MHz: the shader clock
        if (it < 7)
            prof_value(c, it + 8, 5, t);     // (profiling) the tile id
        // top: t's input, offsets and ticket were issued a codec ago and have
        // landed at the last iteration's poll wait; what is still in flight
        // here is that iteration's flush (stores, flag store, super publish),
        // which nothing below reads.  The wait is kept: without it (prologue
        // loads drained before the loop instead) the per-tile top wait fell
        // from 1.8k to 0.3k cycles but the kernels did not get faster (enc
        // 65.6 / dec 68.7 vs 65.3 / 68.3 us, interleaved A/B, profiles/r02_g)
        // -- the waves then wait longer in their look-backs.
        wait_vm_all();
        prof_stamp(c, it, 1);
        if (sp_cur.staged)
            pol.stage_in(ch, sp_cur, o_cur);
        wave_sync();
        // loads for the next tiles, a whole codec ahead of their use: input
        // of tn, the ticket of the tile after it (read after the codec, when
        // its offsets are loaded: they land by the next top); the oldest
        // pending tile's look-back polls.  A tile is thus claimed two
        // iterations before it is coded (three until round 4: the ticket a
        // whole iteration ahead of its offsets load), which matters at the
        // end of a batch: the last tiles go to whichever waves claim them,
        // and the slowest waves then hold them longest.
        const Span sp_nxt = tile_span(in, o_nxt.first(), o_nxt.last(), P::kInCap);
        ch.load(sp_nxt);
        uint32_t kq = kNone;
        if (kpre != kClaimNow)
        {
            kq = kpre;                       // (the prologue's third ticket)
            kpre = kClaimNow;
        }
        else if (tn < nt && tn < stop_fr)
            kq = tk.claim(c);
        LookBack lbo;                        // the oldest pending tile's
        if (pend[0].valid)
        {
            lbo = pend[0].lb();
            lbo.poll(c);
        }
        prof_stamp(c, it, 2);

        // codec of t (LDS only when staged)
        const uint32_t cnt = cnt_of(t);
        uint32_t sz = 0, st = 0;
        bool fast = sp_cur.staged;
        // the pending tiles' outputs to slots (their registers are free
        // for the big-tile or cooperative code that follows)
        auto park = [&]() {
            if constexpr (P::kBig)
#pragma unroll
            for (int i = 0; i < D; ++i)
            {
                if (pend[i].valid && !pend[i].big)
                {
                    const uint32_t kp = big_next % kBigSlots;
                    ++big_next;
                    outs[i].store(big_slot(c, kp), pend[i].total);
                    pend[i].big = kp + 1;
                }
                outs[i].clear();
            }
        };
        if (fast)
        {
            pol.prepare(sp_cur);
            pol.codec(o_cur, cnt, sp_cur, &sz, &st);
#if QH_COOP_VIA_BIG
            // a tile with strings for the whole wave goes the big tiles'
            // way (P::big_sizes runs its cooperative phase): one copy of
            // that code, beside the big-tile path, and the loop keeps the
            // lean kernel's registers
            if (QH_RARE(P::kBig, P::kCoop && pol.coop))
                fast = false;
#else
            if (QH_RARE(P::kBig, P::kCoop && pol.coop))
            {
                park();
                pol.coop_phase(o_cur, 0, cnt, sp_cur, &sz, &st);
            }
#endif
        }
        uint32_t incl = wave_incl_scan(sz);
        uint32_t excl = incl - sz;
        uint32_t total = read_lane(incl, 63);
        fast = fast && total + 64 <= (uint32_t) P::kOutCap;
        uint32_t bigslot = 0;                // (wave-uniform) 1 + the slot
        if constexpr (P::kBig)
        {
            // A big tile (input or output past the stages): its sizes, in
            // staged units, and its output into one of the wave's big-tile slots
            // (P::big_sizes).  When it fits, it is pending like any other tile
            // from here on -- its output copied from the slot when its look-back
            // resolves -- and the wave goes straight on to its next tile.
            if (QH_RARE(P::kBig, !fast))
            {
                // the pending tiles' outputs move to slots first, so that their
                // registers are free for the big tile's codec (the slots hold
                // every tile in flight: kDepth pending + this one)
                park();
                const uint32_t k = big_next % kBigSlots;
                if (pol.big_sizes(cnt, o_cur, sp_cur, sz, st, big_slot(c, k)))
                {
                    bigslot = k + 1;
                    ++big_next;
                }
                incl = wave_incl_scan(sz);
                excl = incl - sz;
                total = read_lane(incl, 63);
                // the next tile's input again: its chunk registers were free
                // through the big tile's codec
                ch.load(sp_nxt);
            }
        }
        prof_stamp(c, it, 3);

        Pending cur;
        cur.valid = false;
        cur.big = 0;
        LookBack lbc;                        // t's publication
        if (fast || bigslot)
        {
            // publish t's aggregate, pack t into the LDS out stage
            cur.valid = true;
            cur.excl = excl;
            cur.stat = st;
            cur.tile = t;
            cur.total = total;
            cur.big = bigslot;
            lbc.start(c, t, total);
            if (fast)
            {
                wave_sync();
                pol.emit(excl, sz, total);
                wave_sync();
            }
        }
        prof_stamp(c, it, 9);
#ifdef QHUFF_PROFILE
        // (profiling only) split the wait: all but the youngest three -- the
        // aggregate store and super add of lb.start, stamp 9 -- then the rest
        __builtin_amdgcn_s_waitcnt(0x0f73);
        prof_stamp(c, it, 10);
#endif

        // the polls (a codec and an emit ago); resolve + store the oldest
        wait_vm_all();
        prof_stamp(c, it, 4);
        // the ticket has landed: the tile after tn, and its offsets
        const uint32_t tnn = tn < nt ? tk.tile_of(kq) : kNone;
        {
            const uint32_t tz = clamp(tnn);
            o_nn.load(in_off, (uint64_t) tz * TS, cnt_of(tz));
        }
        // t's add has returned with the polls: publish its super tile's
        // aggregate if that add completed it -- here, an emit after the add,
        // not at the next iteration's top (look-backs of later super tiles
        // wait on it: encode re-polled the super windows on 1 tile in 3)
        if (cur.valid)
            lbc.super_agg(c);
        if (pend[0].valid)
            flush_at(0, lbo, it);
#pragma unroll
        for (int i = 0; i + 1 < D; ++i)
        {
            pend[i] = pend[i + 1];
            outs[i] = outs[i + 1];
        }
        pend[D - 1] = cur;
        prof_stamp(c, it, 5);

        if (!QH_RARE(P::kBig, !fast))
            outs[D - 1].gather(pol.out_stage());
        else if (bigslot)
            outs[D - 1].clear();             // (its output is in its slot)
        else
        {
            // (rare: a big tile in the lean kernel, or one whose output
            // exceeds a slot) coded out of line after the pending tiles are
            // flushed, so that no tile output is live across the call -- but
            // its sizes first and its aggregate published BEFORE those
            // flushes wait on anything (round 5): the flushes wait on earlier
            // tiles, big ones among them, and a big tile that published only
            // after its own flushes chained every big tile of the batch
            // behind the one before it (the lean kernels' first launch on the
            // QIF corpus: encode ~3 ms against 70 us)
            if constexpr (!P::kBig)
                if (!sp_cur.staged)
                    pol.slow_size(cnt, o_cur, sp_cur, sz, st);
            LookBack lbb;
            lbb.start(c, t, read_lane(wave_incl_scan(sz), 63));
            lbb.super_agg(c);
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (pend[i].valid)
                {
                    LookBack l = pend[i].lb();
                    l.poll(c);
                    flush_at(i, l, ~0u);
                }
            prof_stamp(c, kProfIters - 1, 0);    // (profiling) big tile
            pol.slow_tile(c, t, cnt, o_cur, sp_cur, sz, st, !P::kBig, out,
                          out_off, status, n, lbb);
            prof_stamp(c, kProfIters - 1, 3);
        }
        wave_sync();
        prof_stamp(c, it, 6);

        if (tn >= nt)
            break;
        t = tn;
        tn = tnn;
        o_cur = o_nxt;
        o_nxt = o_nn;
        sp_cur = sp_nxt;
    }
    wait_vm_all();
    prof_stamp(c, kProfIters - 2, 6);        // (profiling) drain start
    // the drain: every pending tile's polls issued together, then each one
    // resolved and stored (one round trip for all of them, not one each:
    // the last waves' drain ends the kernel)
    LookBack ld[D];
#pragma unroll
    for (int i = 0; i < D; ++i)
        if (pend[i].valid)
        {
            ld[i] = pend[i].lb();
            ld[i].poll(c);
        }
#pragma unroll
    for (int i = 0; i < D; ++i)
        if (pend[i].valid)
            flush_at(i, ld[i], ~0u);
#ifdef QHUFF_PROFILE
    wait_vm_all();
    prof_stamp(c, kProfIters - 2, 7);        // (profiling) drain end
    prof_realtime(c, kProfIters - 2, 8);
#endif
    // (The wave claimed until a claim landed past the end, so every ticket
    // of its group is taken, by running waves: see BlockTickets.  A spread
    // launch hands out a prefix of the tiles, one per wave.)
}

}  // namespace qhuff
