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
// Per lane, one string: a position-based decoder over the tile's input,
// staged in LDS as big-endian dwords.  Each step fetches the next 32 bits
// (two LDS dwords + a funnel shift; bits past the string end read as ones,
// the way huff_decode_fast pads its last window, lsqpack.c:5364-5365), looks
// the top 12 bits up in a window table (up to 2 symbols of <= 12 bits), and
// falls back to a canonical length search for codes of 13..30 bits.  Output
// bytes accumulate in a register and land in a per-string LDS arena slot;
// after the workgroup scan + look-back, slots are compacted into an LDS
// output stage and copied out with 16-byte aligned stores.
//
// Persistent grid, static tile assignment, same look-back as the encoder.
#include "qhuff_kernels.h"

namespace qhuff {

constexpr int kDecInCap = 8 * 1024;                    // staged input bytes
// arena slot of string i starts at dword 2i + floor(2 * (rs_i - A) / 5):
// an output is at most 8/5 of its input, so a slot holds the string's output
// words plus one spare dword for the always-store-two emitter
constexpr int kArenaWords = 2 * kTile + 2 * kDecInCap / 5 + 4;

struct DecSmem
{
    uint32_t win[kWinSize];
    uint16_t sorted[257];
    uint32_t off[2][kTile + 1];      // current / next tile offsets
    uint32_t size[kTile];
    uint32_t excl[kTile];
    uint32_t cnt[kBuckets];
    uint16_t perm[kTile];
    uint8_t stat[kTile];
    LdsScratch scr;
    // input stage (big-endian dwords) during decode; output stage after:
    // 16 B pad + at most 8/5 of the staged input + 32 B of copy-out slack
    alignas(16) uint32_t io[((8 * kDecInCap / 5 + 16 + 48) / 16) * 4];
    alignas(16) uint32_t arena[kArenaWords];
    uint32_t junk[2 * 64];           // per-lane junk pair, shared across waves
};

struct DecLds                        // big-endian dwords staged in LDS
{
    const QH_LDS uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
    // the stage has slack past the input: the next dword is always readable
    __device__ __forceinline__ uint32_t dw1(uint32_t i, uint32_t) const
    {
        return w[i + 1];
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
    __device__ __forceinline__ uint32_t dw1(uint32_t i, uint32_t bitend) const
    {
        return (i + 1) * 32 < bitend ? bswap32(w[i + 1]) : 0xffffffffu;
    }
};

// long-code step: canonical search over code lengths 13..30 (uniform table,
// unrolled selects; only runs when some lane of the wave needs it)
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
// stream `src`.  Output goes through `emit(step, val, nbytes)`.  Returns the
// number of output bytes, or -1 for a rejected string.
//
// The loop trip count is uniform across the wave (lanes that finished keep
// computing on clamped positions with their results masked by selects), so
// the body compiles to straight-line VALU + LDS code; only the rare long-code
// step sits behind a wave-uniform branch.
template <class Src, class Emit>
__device__ __forceinline__ int
decode_string(const Src &src, uint32_t bit0, uint32_t bitend,
              const QH_LDS uint32_t *s_win, const QH_LDS uint16_t *s_sorted,
              const LongParams &lp, Emit &emit)
{
    uint32_t abp = bit0;
    bool done = bit0 >= bitend;
    bool bad = false;
    int nout = 0;
    while (__builtin_amdgcn_ballot_w64(!done))
    {
        const uint32_t i = abp >> 5, s = abp & 31;
        const uint32_t rem = bitend - abp;               // >= 1 while !done
        const uint32_t d0 = src.dw(i);
        const uint32_t d1 = src.dw1(i, bitend);
        const uint32_t fs = __builtin_amdgcn_alignbit(d0, d1, (32 - s) & 31);
        uint32_t w = s ? fs : d0;
        w |= rem < 32 ? (0xffffffffu >> (rem & 31)) : 0u; // EOS padding
        const uint32_t e = s_win[w >> (32 - kWinBits)];
        const uint32_t ns = e >> 24, l0 = (e >> 16) & 15, lt = (e >> 20) & 15;
        const bool two = (ns == 2) & (lt <= rem);
        uint32_t c = two ? lt : l0;
        uint32_t val = two ? (e & 0xffff) : (e & 0xff);
        bool eos = false;
        // a code longer than the window cannot fit the remaining bits when
        // rem <= kWinBits: that is the tail (padding), no search needed
        c = (ns == 0) ? 31u : c;
        const bool lng = (ns == 0) & !done & (rem > (uint32_t) kWinBits);
        if (__builtin_amdgcn_ballot_w64(lng))
        {
            uint32_t L;
            uint32_t sym = long_code(w, lp, s_sorted, &L);
            c = lng ? L : c;
            val = lng ? sym : val;
            eos = lng & (sym == 256);
        }
        const uint32_t nb = two ? 2 : 1;
        const bool tail = c > rem;
        // tail: at most 7 bits of EOS prefix may remain (lsqpack.c:5409-5426)
        const bool tail_ok = (rem < 8)
            & ((w >> ((32 - rem) & 31)) == (0xffffffffu >> ((32 - rem) & 31)));
        const bool step = !done & !tail & !eos;
        bad |= !done & ((tail & !tail_ok) | (!tail & eos));
        emit(step, val, nb);
        nout += step ? (int) nb : 0;
        abp += step ? c : 0;
        done = done | !step | (abp >= bitend);
    }
    return bad ? -1 : nout;
}

// arena sink: bytes accumulate little-endian; each step stores the current
// word and the next (a slot has one spare dword), so nothing is left to flush
// and no store depends on a branch.  Lanes not stepping write a junk dword.
struct ArenaEmit
{
    QH_LDS uint32_t *slot;
    QH_LDS uint32_t *junk;             // 2 dwords of this lane
    uint32_t acc, ob, nw;
    __device__ __forceinline__ void operator()(bool step, uint32_t val,
                                               uint32_t nb)
    {
        const uint64_t a64 = (uint64_t) acc | ((uint64_t) val << (8 * ob));
        QH_LDS uint32_t *p = step ? slot + nw : junk;
        p[0] = (uint32_t) a64;
        p[1] = (uint32_t) (a64 >> 32);
        const uint32_t ob2 = ob + nb;
        const bool carry = ob2 >= 4;
        const uint32_t nacc = carry ? (uint32_t) (a64 >> 32) : (uint32_t) a64;
        acc = step ? nacc : acc;
        nw += (step & carry) ? 1 : 0;
        ob = step ? (ob2 & 3) : ob;
    }
};

struct CountEmit
{
    __device__ __forceinline__ void operator()(bool, uint32_t, uint32_t) {}
};

struct GlobalEmit                            // slow path: byte stores
{
    uint8_t *dst;
    uint32_t n;
    __device__ __forceinline__ void operator()(bool step, uint32_t val,
                                               uint32_t nb)
    {
        if (step)
        {
            dst[n++] = (uint8_t) val;
            if (nb == 2)
                dst[n++] = (uint8_t) (val >> 8);
        }
    }
};

constexpr int kDecChunks = kDecInCap / 16 / kTile;      // prefetch regs

__global__ __launch_bounds__(kTile) void
qhuff_decode_kernel(DecArgs a)
{
    __shared__ DecSmem smem;
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    const int tid = threadIdx.x;
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

    // prologue: offsets + input of the first tile
    Prefetch<kDecChunks> pf;
    uint32_t cnt = (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) tile * kTile);
    pf.load_offsets(gin_off, (uint64_t) tile * kTile, cnt);
    pf.store_offsets(sm->off[0], cnt);
    __syncthreads();
    Span sp0 = tile_span(a.in, sm->off[0], cnt, kDecInCap);
    uintptr_t sp_pa = sp0.pa;
    uint32_t sp_n16 = sp0.n16;
    uint32_t sp_staged = sp0.staged;
    if (sp_staged)
    {
        pf.load_chunks(sp_pa, sp_n16);
        pf.store_chunks<true>((QH_LDS u32x4 *) sm->io, sp_n16);
    }
    uint32_t cur = 0;
    int64_t known_tile = -1;                      // see look_back()
    uint64_t known_incl = 0;

    for (;;)
    {
        const QH_LDS uint32_t *off = sm->off[cur];
        const uint64_t s0 = (uint64_t) tile * kTile;
        const uint32_t next = tile + G;
        const bool has_next = next < a.c.n_tiles;
        const uint32_t cnt_n = has_next
            ? (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) next * kTile) : 0;
        if (has_next)
            pf.load_offsets(gin_off, (uint64_t) next * kTile, cnt_n);

        uint32_t key = 0;
        if (tid < (int) cnt)
            key = min((off[tid + 1] - off[tid]) >> 1, (uint32_t) kBuckets - 1);
        const uint32_t my = sort_by_bucket(key, sm->cnt, sm->perm);
        const bool valid = my < cnt;
        const uint32_t A = off[0];
        const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (a.in + off[my]) - sp_pa) : 0;
        const uint32_t re = valid ? (uint32_t) ((uintptr_t) (a.in + off[my + 1]) - sp_pa) : 0;
        const uint32_t slot0 = 2 * my + (uint32_t) ((2ull * (off[my] - A)) / 5);

        // decode (sizes + arena bytes)
        if (valid)
        {
            int r;
            if (a.c.dbg & kDbgNoCodec)
                r = (int) (re - rs);
            else if (sp_staged)
            {
                ArenaEmit em{sm->arena + slot0, sm->junk + 2 * (tid & 63), 0, 0, 0};
                r = decode_string(DecLds{sm->io}, 8 * rs, 8 * re, sm->win,
                                  sm->sorted, a.lp, em);
            }
            else
            {
                CountEmit em;
                r = decode_string(DecGlb{(const QH_GLB uint32_t *) sp_pa},
                                  8 * rs, 8 * re, sm->win, sm->sorted, a.lp, em);
            }
            sm->size[my] = r < 0 ? 0 : (uint32_t) r;
            sm->stat[my] = r < 0 ? QHUFF_DEC_ERROR : QHUFF_DEC_OK;
        }
        if (has_next)
            pf.store_offsets(sm->off[cur ^ 1], cnt_n);
        __syncthreads();

        const uint32_t sz_t = tid < (int) cnt ? sm->size[tid] : 0;
        uint32_t total;
        const uint32_t ex_t = block_excl_scan(sz_t, &sm->scr, &total);
        sm->excl[tid] = ex_t;
        publish_aggregate(a.c, tile, total);
        LbPoll pl;
        if (!(a.c.dbg & kDbgNoLookback))
            look_back_load(a.c, (int64_t) tile - 1, known_tile, known_incl, &pl);
        if (sp_staged)
        {
            // the input stage is dead: zero it as the output stage
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) sm->io;
            const uint32_t n16 = (total + 16 + 15) / 16 + 1;
            for (uint32_t i = tid; i < n16; i += kTile)
                o4[i] = (u32x4){0, 0, 0, 0};
        }
        __syncthreads();

        // next tile's input: issue the loads now, land them after copy-out
        uintptr_t nx_pa = 0;
        uint32_t nx_n16 = 0, nx_staged = 0;
        if (has_next)
        {
            Span t = tile_span(a.in, sm->off[cur ^ 1], cnt_n, kDecInCap);
            nx_pa = t.pa;
            nx_n16 = t.n16;
            nx_staged = t.staged;
            if (nx_staged)
                pf.load_chunks(nx_pa, nx_n16);
        }

        // compaction: arena slot -> output stage at byte 16 + excl
        const uint32_t nout = valid ? sm->size[my] : 0;
        if (sp_staged && nout && !(a.c.dbg & kDbgNoCodec))
        {
            const uint32_t D = 16 + sm->excl[my];
            const uint32_t sh = 8 * (D & 3);
            const uint32_t nwd = (nout + 3) >> 2;
            QH_LDS uint32_t *o = sm->io + (D >> 2);
            const QH_LDS uint32_t *src = sm->arena + slot0;
            for (uint32_t k = 0; k < nwd; ++k)
            {
                uint32_t w = src[k];
                uint32_t vb = nout - 4 * k;
                if (vb < 4)
                    w &= (1u << (8 * vb)) - 1;
                __hip_atomic_fetch_or(&o[k], w << sh, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                if (sh)
                    __hip_atomic_fetch_or(&o[k + 1], w >> (32 - sh),
                                          __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }

        const uint64_t base = (a.c.dbg & kDbgNoLookback) ? (uint64_t) tile << 16
                            : look_back(a.c, tile, total, &sm->scr, pl,
                                        known_tile, known_incl);
        known_tile = tile;                        // this WG's next tile is
        known_incl = base + total;                // tile + G: it knows this
        __syncthreads();

        if (!(a.c.dbg & kDbgNoStore))
        {
            if (sp_staged)
                copy_out(sm->io, a.out + base, total);
            else if (nout)
            {
                GlobalEmit em{a.out + base + sm->excl[my], 0};
                decode_string(DecGlb{(const QH_GLB uint32_t *) sp_pa}, 8 * rs,
                              8 * re, sm->win, sm->sorted, a.lp, em);
            }
            QH_GLB uint32_t *gout_off = glb(a.out_off);
            QH_GLB uint8_t *gstat = glb(a.status);
            if (tid < (int) cnt)
            {
                gout_off[s0 + tid] = (uint32_t) (base + ex_t);
                gstat[s0 + tid] = sm->stat[tid];
            }
            if (tile == a.c.n_tiles - 1 && tid == 0)
                gout_off[a.n] = (uint32_t) (base + total);
        }
        if (!has_next)
            break;
        __syncthreads();
        if (nx_staged)
            pf.store_chunks<true>((QH_LDS u32x4 *) sm->io, nx_n16);
        tile = next;
        cnt = cnt_n;
        sp_pa = nx_pa;
        sp_n16 = nx_n16;
        sp_staged = nx_staged;
        cur ^= 1;
    }
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
