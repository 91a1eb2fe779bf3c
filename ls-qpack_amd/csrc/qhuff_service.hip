// qhuff_service.hip -- the low-latency path: a resident (persistent) kernel
// that serves small encode / decode requests posted by host threads into
// pinned request slots, with no kernel launch, no hipMemcpy and no stream
// synchronisation per request (include/qhuff.h qhuff_svc_*).
//
// Why: the reference codes one literal per call (lsqpack.c:3718, 3795, 4714,
// 4824, 4908 decode; 1983-2119 encode) and a header block holds 10-50 of
// them; a batch launch costs ~21 us device-resident and ~50 us from host
// memory, almost all of it launch, copy and
// synchronisation latency.  Here each wave of the service owns one slot in
// fine-grained host memory and polls its request word; a request is
//   1. coded tile by tile (64 strings) in the wave with the batch kernels'
//      own policies (qhuff_decode_impl.h / qhuff_encode_impl.h: the same
//      staged codec, emit and slow path -- the tiles' bases are a running
//      sum, no look-back): a one-tile request straight from the slot into
//      the slot, a longer one through the slot's device scratch (copied in
//      and out in parallel passes of 16-byte loads),
//   2. completed by a system-scope release and the done word.
// The workgroup's LDS holds both codes' tables (loaded once per launch) and
// one wave region per slot (the union of the decode and encode regions).
//
// Lifetime: a wave leaves when the host raises the stop word, when no wave
// of the service has served a request for idle_ticks (the host relaunches
// on demand), or after life_ticks; every poll checks all three, so the grid
// always drains.
#include "qhuff_decode_impl.h"
#include "qhuff_encode_impl.h"

namespace qhuff {

static_assert(kSvcTileBytes == (uint32_t) kStageCap, "host piece size");

union SvcWave
{
    DecWave d;
    EncWave e;
};

struct SvcSmem
{
    static constexpr bool kMtRep = false;   // (no LDS left for 32 copies)
    uint32_t win[kWinSize + 4];      // decode window table + the hold entry
    uint16_t sorted[257];
    uint16_t long2[kLong2Size];      // decode: long codes by leading ones
    u32x2 enc[257];                  // encode tables (enc_tables_load)
    uint32_t mt[256];
    uint8_t len[256];
    uint32_t quit;                   // a wave saw the service idle: all leave
    SvcWave w[kWaves];
};

__device__ __forceinline__ uint32_t
sys_load(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// a slot header's first 16 bytes in one system-coherent load (sc0 sc1: past
// the caches, as the system-scope atomic loads are), waited for
__device__ __forceinline__ u32x4
poll_hdr(const SvcHdr *h)
{
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=v"(v)
                 : "v"(h)
                 : "memory");
    return v;
}

// 16-byte chunks [0, na) of region a, then [0, nb) of region b, from src
// to dst (two regions of the slot layout, in one pass: one memory round
// trip for up to 8 chunks per lane)
__device__ __forceinline__ void
copy2(const uint8_t *src, uint8_t *dst, uint32_t a, uint32_t na, uint32_t b,
      uint32_t nb)
{
    const uint32_t lane = lane_id();
    const uint32_t n16 = na + nb;
    for (uint32_t k0 = 0; k0 < n16; k0 += 64 * 8)
    {
        u32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
        {
            const uint32_t i = k0 + lane + 64 * j;
            const uint32_t q = i < n16 ? i : 0;
            const uint32_t at = q < na ? a + 16 * q : b + 16 * (q - na);
            v[j] = *(const QH_GLB u32x4 *) (src + at);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
        {
            const uint32_t i = k0 + lane + 64 * j;
            const uint32_t at = i < na ? a + 16 * i : b + 16 * (i - na);
            if (i < n16)
                *(QH_GLB u32x4 *) (dst + at) = v[j];
        }
    }
}

// one request's tiles, in order, in this wave; returns the output bytes
template <class P>
__device__ __forceinline__ uint64_t
serve_tiles(P &pol, const uint8_t *in, const uint32_t *in_off, uint32_t n,
            uint32_t nbytes, uint8_t *out, uint32_t *out_off, uint8_t *status)
{
    const uint32_t lane = lane_id();
    const bool one_tile = n <= P::kTS;
    uint64_t base = 0;
    for (uint32_t s0 = 0; s0 < n; s0 += P::kTS)
    {
        const uint32_t cnt = n - s0 < P::kTS ? n - s0 : P::kTS;
        typename P::Offs o;
        o.load((const QH_GLB uint32_t *) in_off, s0, cnt);
        // one tile (its strings from byte 0, the offsets rebased): the span
        // is known without the offsets, so the offsets and the chunks are
        // loaded together -- over PCIe, one round trip
        const Span sp = one_tile ? Span{(uintptr_t) in, (nbytes + 15) / 16,
                                        nbytes <= (uint32_t) P::kInCap}
                                 : tile_span(in, o.first(), o.last(), P::kInCap);
        Chunks<P::kNch> ch;
        ch.load(sp);
        if (sp.staged)
            pol.stage_in(ch, sp, o);
        wave_sync();
        uint32_t sz = 0, st = 0;
        bool fast = sp.staged;
        if (fast)
        {
            pol.prepare(sp);
            pol.codec(o, cnt, sp, &sz, &st);
            if (P::kCoop && pol.coop)
                pol.coop_phase(o, 0, cnt, sp, &sz, &st);
        }
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t excl = incl - sz;
        const uint32_t total = read_lane(incl, 63);
        fast = fast && total + 64 <= (uint32_t) P::kOutCap;
        if (fast)
        {
            wave_sync();
            pol.emit(excl, sz, total);
            wave_sync();
            TileOut<P::kNch> to;
            to.gather(pol.out_stage());
            to.store(out + base, total);
            if (lane < cnt)
            {
                ((QH_GLB uint32_t *) out_off)[s0 + lane] = (uint32_t) (base + excl);
                if (P::kStatus)
                    ((QH_GLB uint8_t *) status)[s0 + lane] = (uint8_t) st;
            }
            base += total;
        }
        else
            base = pol.slow_tile_at(base, cnt, o, sp, sz, st, out, out_off + s0,
                                    P::kStatus ? status + s0 : nullptr);
        wave_sync();
    }
    if (lane == 0)
        ((QH_GLB uint32_t *) out_off)[n] = (uint32_t) base;
    return base;
}

__global__ __launch_bounds__(64 * kWaves) void
qhuff_service_kernel(SvcArgs a)
{
    __shared__ SvcSmem smem;
    QH_LDS SvcSmem *sm = (QH_LDS SvcSmem *) &smem;
    const int tid = threadIdx.x;
    {
        const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) glb(a.win);
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
        for (int i = tid; i < kWinSize / 4; i += 64 * kWaves)
            sw[i] = gw[i];
        if (tid < 257)
            sm->sorted[tid] = glb(a.sorted)[tid];
        for (int i = tid; i < kLong2Size; i += 64 * kWaves)
            sm->long2[i] = glb(a.long2)[i];
        if (tid == 0)
            sm->win[kHoldIdx] = kHoldEntry;          // (decode)
        enc_tables_load(sm, a.enc, tid);
        if (tid == 0)
            sm->quit = 0;
    }
    __syncthreads();                 // the only workgroup barrier

    const uint32_t lane = lane_id();
    const uint32_t slot = blockIdx.x * (uint32_t) kWaves + (tid >> 6);
    uint8_t *sb = a.slots + (uint64_t) slot * kSvcSlotBytes;
    SvcHdr *h = (SvcHdr *) sb;
    uint8_t *scr = a.scratch + (uint64_t) slot * kSvcScratchBytes;
    QH_LDS SvcWave *wv = &sm->w[tid >> 6];

    // a request posted while no service ran (req != done) is served first
    uint32_t last = __builtin_amdgcn_readfirstlane(sys_load(&h->done));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0;; ++it)
    {
        // one PCIe round trip per poll: the request word and its fields
        const u32x4 hd = poll_hdr(h);
        const uint32_t req = __builtin_amdgcn_readfirstlane(hd.x);
        if (req != last)
        {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            if (lane == 0)                   // busy: nobody leaves for idle
                __hip_atomic_fetch_max((unsigned long long *) a.active,
                                       (unsigned long long) __builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t n = __builtin_amdgcn_readfirstlane(hd.y);
            const uint32_t in_bytes = __builtin_amdgcn_readfirstlane(hd.z);
            const uint32_t op = __builtin_amdgcn_readfirstlane(hd.w) & 0xff;
            const uint32_t mode = __builtin_amdgcn_readfirstlane(hd.w) >> 8;
            // (the host checks n, in_bytes and the offsets; these bounds only
            // keep a corrupt slot inside its own memory)
            const uint32_t nn = n < kSvcMaxStrings ? n : kSvcMaxStrings;
            const uint32_t nb = in_bytes < kSvcInCap ? in_bytes : kSvcInCap;
            // One staged tile: straight from the slot and into it (its loads
            // in one PCIe round trip, its stores waited for once, at the
            // end).  More tiles: through the device scratch -- a tile's loads
            // would otherwise wait for the previous tile's stores to host
            // memory (loads and stores share vmcnt, in order).
            const bool one = nn <= (uint32_t) kWT && nb <= (uint32_t) kStageCap;
            uint8_t *io = one ? sb : scr;
            if (!one)
            {
                copy2(sb, scr, kSvcInOffAt, ((nn + 1) * 4 + 15) / 16, kSvcInAt,
                      (nb + 15) / 16);
                // the copies land before other lanes of the wave read them
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            const uint8_t *in = io + kSvcInAt;
            const uint32_t *in_off = (const uint32_t *) (io + kSvcInOffAt);
            uint8_t *out = io + kSvcOutAt;
            uint32_t *out_off = (uint32_t *) (io + kSvcOutOffAt);
            uint64_t total;
            if (op == kSvcOpEncode)
            {
                EncPolicyT<SvcSmem> pol;
                pol.in = in;
                pol.mode = mode;
                pol.sm = sm;
                pol.wv = &wv->e;
                pol.dense = false;
                total = serve_tiles(pol, in, in_off, nn, nb, out, out_off,
                                    nullptr);
            }
            else
            {
                DecPolicyT<SvcSmem> pol{in, sm, &wv->d, 0};
                total = serve_tiles(pol, in, in_off, nn, nb, out, out_off,
                                    io + kSvcStatusAt);
            }
            if (!one)
            {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                const uint32_t tot = (uint32_t) total;
                copy2(scr, sb, kSvcOutOffAt, ((nn + 1) * 4 + 15) / 16,
                      kSvcStatusAt, (nn + 15) / 16);
                copy2(scr, sb, kSvcOutAt, (tot + 15) / 16, 0, 0);
            }
            // every output store of the wave completed (system scope), then
            // the done word
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (lane == 0)
            {
                __hip_atomic_store(&h->total, (uint32_t) total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&h->done, req, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_fetch_max((unsigned long long *) a.active,
                                       (unsigned long long) __builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            last = req;
            it = 0;
            continue;
        }
        // Leaving: the waves of a workgroup leave together (a wave that left
        // alone would strand its slot until the last wave had gone idle --
        // tens of ms for a call that picked that slot while others were
        // busy); a request that arrives after its wave's last poll is
        // served by the next launch (the waiting host starts one when it
        // finds the service stream idle).
        if (__builtin_amdgcn_readfirstlane(*(volatile QH_LDS uint32_t *) &sm->quit))
            break;
        if (it % 16 != 15)                   // stop word and clock: every 16th
            continue;
        if (__builtin_amdgcn_readfirstlane(sys_load(&a.ctl[0])))
            break;
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        const uint64_t act = __hip_atomic_load((unsigned long long *) a.active,
                                               __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t since = act > t0 ? act : t0;
        if (now - since > a.idle_ticks || now - t0 > a.life_ticks)
        {
            *(volatile QH_LDS uint32_t *) &sm->quit = 1;
            break;
        }
    }
}

hipError_t
launch_service(const SvcArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_service_kernel, dim3(grid), dim3(64 * kWaves), 0,
                       st, a);
    return hipGetLastError();
}

int
service_waves_per_block()
{
    return kWaves;
}

size_t
service_lds_bytes()
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(qhuff_service_kernel))
            != hipSuccess)
        return 0;
    return fa.sharedSizeBytes;
}

}  // namespace qhuff
