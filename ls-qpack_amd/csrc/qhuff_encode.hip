// qhuff_encode.hip -- batch Huffman encode kernel (gfx950).
//
// Reference path:
//   E1 qenc_enc_str_size   lsqpack.c:5198-5210  -> sizing pass below
//   E2 qenc_huffman_enc    lsqpack.c:5085-5195  -> packing pass below
//   E3 lsqpack_enc_enc_str lsqpack.c:839-876    -> LITERAL modes (H bit,
//                          prefixed length, strict-< Huffman-vs-raw choice)
//
// Persistent grid: every workgroup is resident and walks tiles t = blockIdx.x,
// blockIdx.x + gridDim.x, ... (no ticket atomic).  Per tile of 256 strings:
//   1. stage the tile's packed input bytes into LDS (coalesced 16-B loads);
//   2. counting-sort the strings by length so each wave runs similar lengths;
//   3. sizing pass per lane (code-length sum out of an LDS table);
//   4. workgroup scan -> tile-local output offsets; publish the aggregate;
//   5. packing pass per lane into a zeroed LDS output stage (MSB-first bit
//      accumulator, big-endian words OR-ed in, EOS-prefix padding);
//   6. look-back for the tile's global output base (its latency overlaps the
//      packing of step 5 in the other resident workgroups);
//   7. shifted copy-out with 16-byte aligned global stores; out_off stores.
// Tiles whose input or output does not fit the LDS stages take the same steps
// with global reads / per-lane global writes (correct, slower).
#include "qhuff_kernels.h"

namespace qhuff {


// source of aligned input dwords: LDS stage or global
struct EncLds
{
    const QH_LDS uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};
struct EncGlb
{
    const QH_GLB uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};

// MSB-first bit packer.  Words are flushed as big-endian dwords at 4-byte
// aligned positions; `lo`..`hi` are the bytes this string owns.
struct PackLds                               // OR into a zeroed LDS stage
{
    QH_LDS uint32_t *stage;
    __device__ __forceinline__ void word(uint32_t wpos, uint32_t be,
                                         uint32_t, uint32_t) const
    {
        __hip_atomic_fetch_or(&stage[wpos >> 2], bswap32(be),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
};

struct PackGlb                               // direct global stores
{
    uint8_t *out;                            // 4-byte aligned
    __device__ __forceinline__ void word(uint32_t wpos, uint32_t be,
                                         uint32_t lo, uint32_t hi) const
    {
        if (wpos >= lo && wpos + 4 <= hi)
            *(QH_GLB uint32_t *) (out + wpos) = bswap32(be);
        else
            for (int k = 0; k < 4; ++k)
            {
                uint32_t p = wpos + k;
                if (p >= lo && p < hi)
                    out[p] = (uint8_t) (be >> (24 - 8 * k));
            }
    }
};

template <class Sink>
struct Packer
{
    Sink sink;
    uint64_t acc;          // pending bits, left-aligned
    uint32_t nbits;        // bits in acc, counting the lead-in bytes
    uint32_t wpos, lo, hi;

    __device__ __forceinline__ void init(uint32_t start, uint32_t end)
    {
        lo = start;
        hi = end;
        wpos = start & ~3u;
        nbits = 8u * (start & 3);
        acc = 0;
    }
    __device__ __forceinline__ void put(uint32_t code, uint32_t len)
    {
        // len == 0 is a no-op (masked byte)
        const uint64_t v = len ? (uint64_t) code << (64 - nbits - len) : 0;
        acc |= v;
        nbits += len;
        if (nbits >= 32)
        {
            sink.word(wpos, (uint32_t) (acc >> 32), lo, hi);
            acc <<= 32;
            nbits -= 32;
            wpos += 4;
        }
    }
    // EOS-prefix padding to a byte boundary, then flush (lsqpack.c:5171-5189)
    __device__ __forceinline__ void finish()
    {
        uint32_t pad = (8 - (nbits & 7)) & 7;
        acc |= (uint64_t) ((1u << pad) - 1) << (64 - nbits - pad);
        nbits += pad;
        while (nbits > 0)
        {
            sink.word(wpos, (uint32_t) (acc >> 32), lo, hi);
            acc <<= 32;
            nbits = nbits > 32 ? nbits - 32 : 0;
            wpos += 4;
        }
    }
};

// HPACK prefixed-integer byte count (lsqpack_val2len, lsqpack.c:767-783)
__device__ __forceinline__ uint32_t
int_len(uint32_t v, uint32_t prefix)
{
    uint32_t mask = (1u << prefix) - 1;
    if (v < mask)
        return 1;
    v -= mask;
    uint32_t n = 2;
    while (v >= 128)
    {
        v >>= 7;
        ++n;
    }
    return n;
}

// valid-byte mask (4 bits) of dword d for a string [rs, re), re > rs
__device__ __forceinline__ uint32_t
byte_mask(uint32_t d, uint32_t d0, uint32_t dl, uint32_t rs, uint32_t re)
{
    uint32_t m = 0xfu;
    m &= (d == d0) ? (0xfu << (rs & 3)) : 0xfu;
    m &= (d == dl) ? (0xfu >> (3 - ((re - 1) & 3))) : 0xfu;
    return m;
}

// sum of code lengths over bytes [rs, re) (positions relative to the source):
// four independent LDS lookups per dword, masked and summed with v_sad_u8
template <class Src>
__device__ __forceinline__ uint32_t
code_bits(const Src &src, uint32_t rs, uint32_t re, const QH_LDS uint8_t *s_len)
{
    uint32_t bits = 0;
    if (re == rs)
        return 0;
    const uint32_t d0 = rs >> 2, dl = (re - 1) >> 2;
    for (uint32_t d = d0; d <= dl; ++d)
    {
        const uint32_t w = src.dw(d);
        const uint32_t l0 = s_len[w & 0xff];
        const uint32_t l1 = s_len[(w >> 8) & 0xff];
        const uint32_t l2 = s_len[(w >> 16) & 0xff];
        const uint32_t l3 = s_len[w >> 24];
        const uint32_t m = byte_mask(d, d0, dl, rs, re);
        // expand the 4-bit mask to bytes: 0x000000ff per set bit
        const uint32_t bm = (m & 1 ? 0xffu : 0u) | (m & 2 ? 0xff00u : 0u)
                          | (m & 4 ? 0xff0000u : 0u) | (m & 8 ? 0xff000000u : 0u);
        const uint32_t packed = l0 | (l1 << 8) | (l2 << 16) | (l3 << 24);
        bits = __builtin_amdgcn_sad_u8(packed & bm, 0u, bits);
    }
    return bits;
}

template <class Src, class Sink>
__device__ __forceinline__ void
pack_string(const Src &src, uint32_t rs, uint32_t re, bool raw,
            const QH_LDS u32x2 *s_enc, Packer<Sink> &pk)
{
    if (re == rs)
        return;
    const uint32_t d0 = rs >> 2, dl = (re - 1) >> 2;
    for (uint32_t d = d0; d <= dl; ++d)
    {
        const uint32_t w = src.dw(d);
        const uint32_t m = byte_mask(d, d0, dl, rs, re);
        // unconditional lookups (independent LDS reads), then masked puts
        u32x2 e[4];
#pragma unroll
        for (int b = 0; b < 4; ++b)
        {
            const uint32_t c = (w >> (8 * b)) & 0xff;
            const u32x2 t = s_enc[c];            // always read: no branch
            e[b].x = raw ? c : t.x;
            e[b].y = raw ? 8u : t.y;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b)
            pk.put(e[b].x, (m >> b) & 1 ? e[b].y : 0u);
    }
}

// literal framing (lsqpack.c:852-854, 862-864, 819-836): H bit + prefixed
// length, then the payload
template <class Src, class Sink>
__device__ __forceinline__ void
emit_string(const Src &src, uint32_t rs, uint32_t re, uint32_t mode,
            bool huff, uint32_t plen, const QH_LDS u32x2 *s_enc,
            Packer<Sink> &pk)
{
    if (mode)
    {
        uint32_t mask = (1u << mode) - 1, first = huff ? (1u << mode) : 0;
        if (plen < mask)
            pk.put(first | plen, 8);
        else
        {
            pk.put(first | mask, 8);
            uint32_t v = plen - mask;
            while (v >= 128)
            {
                pk.put(0x80 | (v & 0x7f), 8);
                v >>= 7;
            }
            pk.put(v, 8);
        }
    }
    pack_string(src, rs, re, !huff, s_enc, pk);
    pk.finish();
}

constexpr int kEncInCapL = 12 * 1024;       // staged input bytes per tile
constexpr int kEncOutCapL = 12 * 1024;      // staged output bytes per tile

struct EncSmem
{
    u32x2 enc[257];
    uint8_t len[256];
    uint32_t off[2][kTile + 1];      // current / next tile offsets
    uint32_t size[kTile];
    uint32_t excl[2][kTile];         // tile offsets, by tile parity
    uint32_t cnt[kBuckets];
    uint16_t perm[kTile];
    LdsScratch scr;
    alignas(16) uint32_t in[kEncInCapL / 4 + 4];
    alignas(16) uint32_t out[2][(kEncOutCapL + 64) / 4];  // 16 B pad in front
};

constexpr int kEncChunks = (kEncInCapL / 16 + kLoadThreads - 1) / kLoadThreads;

// per-string sizing result
struct EncSize
{
    uint32_t size, plen;
    bool huff;
};

template <class Src>
__device__ __forceinline__ EncSize
size_string(const EncArgs &a, const Src &src, uint32_t rs, uint32_t re,
            const QH_LDS uint8_t *s_len)
{
    EncSize z;
    const uint32_t len = re - rs;
    const uint32_t hb = (a.c.dbg & kDbgNoCodec) ? len
                      : (code_bits(src, rs, re, s_len) + 7) >> 3;
    z.huff = true;
    z.plen = 0;
    if (a.mode == 0)
        z.size = hb;
    else
    {
        z.huff = hb < len;                       // strict <, lsqpack.c:848
        z.plen = z.huff ? hb : len;
        z.size = int_len(z.plen, a.mode) + z.plen;
    }
    return z;
}

// the unit whose look-back / copy-out is deferred to the next iteration
struct EncDeferred
{
    uint32_t tile, lo, hi;     // strings [lo, hi) of `tile`
    uint32_t total;            // output bytes of the unit
    uint32_t unit_off;         // output bytes of the tile's earlier units
    uint32_t par;              // stage parity holding its output
    uint32_t staged_out;
    bool first, last;          // first / last unit of its tile
};

// look-back wave: the deferred unit's output base (see the decoder's
// resolve_unit_base)
__device__ __forceinline__ uint64_t
enc_resolve_unit_base(const Coord &c, const EncDeferred &df, int64_t *known_tile,
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

// every thread: copy-out and out_off of the deferred unit; a unit whose
// output did not fit the stage is packed again by every lane straight to
// global memory (input read from global)
__device__ __forceinline__ void
enc_finish(const EncArgs &a, QH_LDS EncSmem *sm, const EncDeferred &df,
           uint64_t base)
{
    const int tid = threadIdx.x;
    if (a.c.dbg & kDbgNoStore)
        return;
    const uint32_t ucnt = df.hi - df.lo;
    const uint64_t s0 = (uint64_t) df.tile * kTile + df.lo;
    QH_GLB uint32_t *gout_off = glb(a.out_off);
    if (df.staged_out)
        copy_out(sm->out[df.par], a.out + base, df.total);
    else if (tid < (int) ucnt)
    {
        const QH_GLB uint32_t *gin_off = glb(a.in_off);
        const uint32_t o0 = gin_off[s0 + tid], o1 = gin_off[s0 + tid + 1];
        const uintptr_t pa = (uintptr_t) (a.in + o0) & ~(uintptr_t) 3;
        const uint32_t rs = (uint32_t) ((uintptr_t) (a.in + o0) - pa);
        const uint32_t re = rs + (o1 - o0);
        EncGlb src{(const QH_GLB uint32_t *) pa};
        EncSize z = size_string(a, src, rs, re, sm->len);
        const uint32_t adj = (uint32_t) ((uintptr_t) a.out & 3);
        Packer<PackGlb> pk;
        pk.sink.out = a.out - adj;
        const uint32_t p0 = adj + (uint32_t) base + sm->excl[df.par][tid];
        pk.init(p0, p0 + z.size);
        emit_string(src, rs, re, a.mode, z.huff, z.plen, sm->enc, pk);
    }
    if (tid < (int) ucnt)
        gout_off[s0 + tid] = (uint32_t) (base + sm->excl[df.par][tid]);
    if (df.last && df.tile == a.c.n_tiles - 1 && tid == 0)
        gout_off[a.n] = (uint32_t) (base + df.total);
    stamp(a.c, df.tile, 13);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3, 3))) void
qhuff_encode_kernel(EncArgs a)
{
    __shared__ EncSmem smem;
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_claim;           // tile after `next` (look-back wave)
    __shared__ uint32_t s_red;             // next unit's end (unit_vote)
    __shared__ unsigned long long s_acc;   // tile aggregate accumulator
    QH_LDS EncSmem *sm = (QH_LDS EncSmem *) &smem;
    QH_LDS uint32_t *red = (QH_LDS uint32_t *) &s_red;
    const int tid = threadIdx.x;
    const bool lbw = is_lb_wave();
    if (a.c.dbg & kDbgCensus)
    {
        census(a.c);
        return;
    }

    const QH_GLB u32x2 *genc = (const QH_GLB u32x2 *) a.enc;
    {
        const u32x2 e_t = genc[tid];
        sm->enc[tid] = e_t;
        sm->len[tid] = (uint8_t) e_t.y;
    }
    if (tid == 0)
    {
        sm->enc[256] = genc[256];
        s_acc = 0;
        s_red = 1;
    }

    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    uint32_t tile, next;
    claim_first(a.c, &tile, &next);
    if (tile >= a.c.n_tiles)
        return;

    // prologue: offsets, first unit and its input
    Prefetch<kEncChunks> pf;
    uint32_t cnt = (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) tile * kTile);
    pf.load_offsets(gin_off, (uint64_t) tile * kTile, cnt);
    pf.store_offsets(sm->off[0], cnt);
    __syncthreads();
    unit_vote(a.in, sm->off[0], 0, cnt, kEncInCapL, red);
    __syncthreads();
    uint32_t lo = 0, hi = s_red;
    Span sp0 = unit_span(a.in, sm->off[0], lo, hi, kEncInCapL);
    uintptr_t sp_pa = sp0.pa;
    uint32_t sp_n16 = sp0.n16;
    uint32_t sp_staged = sp0.staged;
    if (sp_staged)
    {
        pf.load_chunks(sp_pa, sp_n16);
        pf.store_chunks<false>((QH_LDS u32x4 *) sm->in, sp_n16);
    }
    uint32_t cur = 0, par = 0;
    uint32_t unit_off = 0;
    int64_t known_tile = -1;
    uint64_t known_incl = 0, tile_base = 0;
    bool pending = false;
    EncDeferred df = {0, 0, 0, 0, 0, 0, 0, false, false};

    for (;;)
    {
        const QH_LDS uint32_t *off = sm->off[cur];
        const bool last = hi == cnt;
        const bool has_next = next < a.c.n_tiles;
        const bool more = !last || has_next;
        const uint32_t lo_n = last ? 0 : hi;
        const uint32_t cnt_n = !last ? cnt : has_next
            ? (uint32_t) min((uint64_t) kTile, a.n - (uint64_t) next * kTile) : 0;
        uint32_t claimed = a.c.n_tiles;
        if (tid == kBlock - 64 && last && has_next)
            claimed = claim_tile(a.c, next);      // consumed after sizing
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

        // 1. length sort + sizing (E1 / the framing choice of E3); each
        //    wave adds its byte total to the tile aggregate at once
        const uint32_t ucnt = hi - lo;
        uint32_t key = 0;
        if (tid < (int) ucnt)
            key = min((off[lo + tid + 1] - off[lo + tid]) >> 1,
                      (uint32_t) kBuckets - 1);
        const uint32_t my = sort_by_bucket(key, sm->cnt, sm->perm);

        const bool valid = my < ucnt;
        const uint32_t si = lo + (valid ? my : 0);
        const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (a.in + off[si]) - sp_pa) : 0;
        const uint32_t re = valid ? (uint32_t) ((uintptr_t) (a.in + off[si + 1]) - sp_pa) : 0;
        EncSize z = {0, 0, true};
        if (valid)
        {
            z = sp_staged ? size_string(a, EncLds{sm->in}, rs, re, sm->len)
                          : size_string(a, EncGlb{(const QH_GLB uint32_t *) sp_pa},
                                        rs, re, sm->len);
            sm->size[my] = z.size;
        }
        publish_wave_total(a.c, tile, valid ? z.size : 0u, last,
                           (QH_LDS unsigned long long *) &s_acc);
        if (threadIdx.x < 64)
            stamp(a.c, tile, 2);

        // look-back wave: the deferred unit's base
        if (lbw)
            stamp(a.c, tile, 5);
        if (pending && lbw)
        {
            const uint64_t b = enc_resolve_unit_base(a.c, df, &known_tile,
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
            unit_vote(a.in, off_n, lo_n, cnt_n, kEncInCapL, red);

        // 2. scan in string order, clear this parity's stage; next loads
        const uint32_t sz_t = tid < (int) ucnt ? sm->size[tid] : 0;
        uint32_t total;
        const uint32_t ex_t = block_excl_scan(sz_t, &sm->scr, &total);
        const uint32_t hi_n = s_red;
        sm->excl[par][tid] = ex_t;
        const bool staged_out = total + 64 <= (uint32_t) kEncOutCapL;
        if (staged_out)
        {
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) sm->out[par];
            const uint32_t n16 = (total + 16 + 15) / 16 + 1;
            for (uint32_t i = tid; i < n16; i += kBlock)
                o4[i] = (u32x4){0, 0, 0, 0};
        }
        uintptr_t nx_pa = 0;
        uint32_t nx_n16 = 0, nx_staged = 0;
        if (more)
        {
            Span t = unit_span(a.in, off_n, lo_n, hi_n, kEncInCapL);
            nx_pa = t.pa;
            nx_n16 = t.n16;
            nx_staged = t.staged;
            if (nx_staged)
                pf.load_chunks(nx_pa, nx_n16);
        }
        __syncthreads();

        // 3. the deferred unit leaves (other parity); pack (E2 / E3) this
        //    unit into its parity of the stage
        if (pending)
            enc_finish(a, sm, df, s_base);
        const uint32_t myex = valid ? sm->excl[par][my] : 0;
        if (staged_out && valid && !(a.c.dbg & kDbgNoCodec))
        {
            Packer<PackLds> pk;
            pk.sink.stage = sm->out[par];
            pk.init(16 + myex, 16 + myex + z.size);
            if (sp_staged)
                emit_string(EncLds{sm->in}, rs, re, a.mode, z.huff, z.plen,
                            sm->enc, pk);
            else
                emit_string(EncGlb{(const QH_GLB uint32_t *) sp_pa}, rs, re,
                            a.mode, z.huff, z.plen, sm->enc, pk);
        }
        df.tile = tile;
        df.lo = lo;
        df.hi = hi;
        df.total = total;
        df.unit_off = unit_off;
        df.par = par;
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
            pf.store_chunks<false>((QH_LDS u32x4 *) sm->in, nx_n16);
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
        par ^= 1;
    }
    if (lbw)
    {
        const uint64_t b = enc_resolve_unit_base(a.c, df, &known_tile,
                                                 &known_incl, &tile_base);
        if ((tid & 63) == 0)
            s_base = b;
    }
    __syncthreads();
    enc_finish(a, sm, df, s_base);
}

hipError_t
launch_encode(const EncArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_encode_kernel, dim3(grid), dim3(kBlock), 0, st, a);
    return hipGetLastError();
}

hipError_t
encode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_encode_kernel),
        kBlock, 0);
}

size_t
encode_lds_bytes()
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(qhuff_encode_kernel))
            != hipSuccess)
        return 0;
    return fa.sharedSizeBytes;
}

}  // namespace qhuff
