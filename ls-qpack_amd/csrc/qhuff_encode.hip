// qhuff_encode.hip -- batch Huffman encode kernel (gfx950).
//
// Reference path:
//   E1 qenc_enc_str_size   lsqpack.c:5198-5210  -> sizing pass below
//   E2 qenc_huffman_enc    lsqpack.c:5085-5195  -> packing pass below
//   E3 lsqpack_enc_enc_str lsqpack.c:839-876    -> LITERAL modes (H bit,
//                          prefixed length, strict-< Huffman-vs-raw choice)
//
// One string per lane, one 64-string tile per wave (qhuff_device.h).  Per
// tile:
//   1. the tile's packed input bytes sit in the wave's LDS input stage
//      (coalesced 16-B loads issued one tile ahead);
//   2. sizing pass per lane (code-length sum out of an LDS table), the
//      Huffman-or-raw choice of the literal modes;
//   3. wave scan -> tile-local output offsets; aggregate published and the
//      first look-back window polled at once;
//   4. packing pass per lane into the zeroed LDS output stage (MSB-first bit
//      accumulator, big-endian words, EOS-prefix padding);
//   5. look-back for the tile's global output base; shifted copy-out with
//      16-byte aligned global stores; out_off stores.
// Tiles whose input or output does not fit the LDS stages take the same
// steps with global reads / per-lane global writes (correct, slower).
#include "qhuff_kernels.h"

namespace qhuff {

constexpr int kEncWaves = 16;                 // waves per workgroup
constexpr int kEncInCap = 3072;               // staged input bytes per tile
constexpr int kEncOutCap = 3072;              // output stage bytes per tile
constexpr int kEncChunks = kEncInCap / 16 / 64;
constexpr int kEncOutChunks = 3;                 // covers a stage of 3072 B

struct EncWave                                // one wave's private LDS region
{
    alignas(16) uint32_t in[kEncInCap / 4 + 4];
    alignas(16) uint32_t out[kEncOutCap / 4];     // 16 B pad in front
};

struct EncSmem
{
    u32x2 enc[257];
    uint8_t len[256];
    EncWave w[kEncWaves];
};

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
struct PackLds                               // into a zeroed LDS stage
{
    QH_LDS uint32_t *stage;
    // a dword this string owns whole is stored; one it shares with a
    // neighbour (its first / last) is OR-ed in
    __device__ __forceinline__ void word(uint32_t wpos, uint32_t be,
                                         uint32_t lo, uint32_t hi) const
    {
        if (wpos >= lo && wpos + 4 <= hi)
            stage[wpos >> 2] = bswap32(be);
        else
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


__global__ __launch_bounds__(64 * kEncWaves) void
qhuff_encode_kernel(EncArgs a)
{
    __shared__ EncSmem smem;
    QH_LDS EncSmem *sm = (QH_LDS EncSmem *) &smem;
    const int tid = threadIdx.x;
    {
        const QH_GLB u32x2 *genc = (const QH_GLB u32x2 *) a.enc;
        if (tid < 257)
        {
            const u32x2 e = genc[tid];
            sm->enc[tid] = e;
            if (tid < 256)
                sm->len[tid] = (uint8_t) e.y;
        }
        clear_next_launch(a.c);
    }
    __syncthreads();                 // the only workgroup barrier

    const uint32_t lane = lane_id();
    QH_LDS EncWave *wv = &sm->w[tid >> 6];
    QH_LDS uint32_t *stage = wv->in;
    QH_LDS uint32_t *ostage = wv->out;
    const QH_GLB uint32_t *gin_off = glb(a.in_off);
    QH_GLB uint32_t *gout_off = glb(a.out_off);
    const uint32_t n_waves = gridDim.x * kEncWaves;
    const uint32_t gid = wave_gid(kEncWaves);
    const uint32_t nt = a.c.n_tiles;
    const uint32_t dbg = a.c.dbg;

    auto tile_cnt = [&](uint32_t t) -> uint32_t {
        return (uint32_t) min((uint64_t) kWT, a.n - (uint64_t) t * kWT);
    };

    // Tiles are claimed just in time: a wave claims its next tile only when
    // it is about to code it, so claim order is processing order and a
    // look-back only ever waits on tiles whose codec is already running.
    // The claim -> offsets -> input latency of one wave hides under the
    // codec work of the other waves on its SIMD.
    PhaseClock clk;
    clk.init(dbg);
    for (;;)
    {
        const uint32_t t = claim_tile(a.c, gid, n_waves);
        clk.lap(0);
        if (t >= nt)
            break;
        const uint32_t cnt = tile_cnt(t);
        TileOffs to;
        to.load(gin_off, (uint64_t) t * kWT, cnt);
        const Span sp = tile_span(a.in, to.first(), to.last(), kEncInCap);
        if (sp.staged)
        {
            Chunks<kEncChunks> ch;
            ch.load(sp);
            ch.store<false>((QH_LDS u32x4 *) stage, sp.n16);
        }
        wave_sync();
        clk.lap(1);

        // 1. sizing (E1 / the framing choice of E3)
        const bool valid = lane < cnt;
        const uint32_t rs = valid ? (uint32_t) ((uintptr_t) (a.in + to.o0) - sp.pa) : 0;
        const uint32_t re = valid ? (uint32_t) ((uintptr_t) (a.in + to.o1) - sp.pa) : 0;
        EncSize z = {0, 0, true};
        if (valid)
            z = sp.staged ? size_string(a, EncLds{stage}, rs, re, sm->len)
                          : size_string(a, EncGlb{(const QH_GLB uint32_t *) sp.pa},
                                        rs, re, sm->len);
        const uint32_t incl = wave_incl_scan(z.size);
        const uint32_t excl = incl - z.size;
        clk.lap(2);
        const uint32_t total = read_lane(incl, 63);

        // 2. publish the aggregate, issue the first look-back poll
        LookBack lb;
        if (!(dbg & kDbgNoLookback))
            lb.start(a.c, t, total);
        clk.lap(3);

        // 3. pack (E2 / E3) into the zeroed output stage
        const bool staged_out = total + 64 <= (uint32_t) kEncOutCap;
        if (staged_out)
        {
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) ostage;
            const uint32_t n16 = (total + 16 + 15) / 16 + 1;
            for (uint32_t i = lane; i < n16; i += 64)
                o4[i] = (u32x4){0, 0, 0, 0};
        }
        wave_sync();
        if (staged_out && valid && !(dbg & kDbgNoCodec))
        {
            Packer<PackLds> pk;
            pk.sink.stage = ostage;
            pk.init(16 + excl, 16 + excl + z.size);
            if (sp.staged)
                emit_string(EncLds{stage}, rs, re, a.mode, z.huff, z.plen,
                            sm->enc, pk);
            else
                emit_string(EncGlb{(const QH_GLB uint32_t *) sp.pa}, rs, re,
                            a.mode, z.huff, z.plen, sm->enc, pk);
        }
        wave_sync();

        clk.lap(4);

        // 4. output base
        const uint64_t base = (dbg & kDbgNoLookback) ? (uint64_t) t << 13
                            : lb.finish(a.c);
        clk.lap(5);

        // 5. copy-out
        CopyOut<kEncOutChunks> co;
        if (staged_out)
            co.gather(ostage, a.out + base, total);
        if (!(dbg & kDbgNoStore))
        {
            if (staged_out)
                co.store();
            else if (valid && !(dbg & kDbgNoCodec))
            {
                // output larger than the stage: pack straight to global
                const uint32_t adj = (uint32_t) ((uintptr_t) a.out & 3);
                Packer<PackGlb> pk;
                pk.sink.out = a.out - adj;
                const uint32_t p0 = adj + (uint32_t) base + excl;
                pk.init(p0, p0 + z.size);
                if (sp.staged)
                    emit_string(EncLds{stage}, rs, re, a.mode, z.huff, z.plen,
                                sm->enc, pk);
                else
                    emit_string(EncGlb{(const QH_GLB uint32_t *) sp.pa}, rs, re,
                                a.mode, z.huff, z.plen, sm->enc, pk);
            }
            const uint64_t s0 = (uint64_t) t * kWT;
            if (valid)
                gout_off[s0 + lane] = (uint32_t) (base + excl);
            if (t == nt - 1 && lane == 0)
                gout_off[a.n] = (uint32_t) (base + total);
        }
        wave_sync();
        clk.lap(6);
    }
    clk.flush(a.c.err);
}

hipError_t
launch_encode(const EncArgs &a, uint32_t grid, hipStream_t st)
{
    hipLaunchKernelGGL(qhuff_encode_kernel, dim3(grid), dim3(64 * kEncWaves),
                       0, st, a);
    return hipGetLastError();
}

hipError_t
encode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_encode_kernel),
        64 * kEncWaves, 0);
}

int
encode_waves_per_block()
{
    return kEncWaves;
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
