// qhuff.hip -- MI355X (gfx950) QPACK Huffman string-literal codec: kernels
// and the C-ABI declared in include/qhuff.h.
//
// Hot path:
//   E1 qenc_enc_str_size  lsqpack.c:5198  -> sizing pass of qhuff_encode_tile
//   E2 qenc_huffman_enc   lsqpack.c:5085  -> packing pass of qhuff_encode_tile
//   E3 lsqpack_enc_enc_str lsqpack.c:839  -> LITERAL modes of the same kernel
//   D1/D2 lsqpack_huff_decode -> huff_decode_fast, lsqpack.c:3524/5243
//   D3 accept/reject rule                 -> qhuff_decode_tile
//
// Both kernels are single-pass tile kernels: a workgroup takes a tile of 256
// consecutive strings (one string per lane), stages the tile's packed input
// bytes into LDS with coalesced 16-byte loads, runs the per-string serial
// codec out of LDS tables, computes its output offsets with a workgroup
// prefix scan, and obtains the tile's global output base with a decoupled
// look-back over per-tile flags (tiles are handed out in order by an atomic
// ticket, so a tile only ever waits on tiles already running).  Output is
// compacted in one pass: no second read of the input, no separate scan
// kernel.  See DESIGN.md for the data layout and roofline accounting.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "../../include/qhuff.h"
#include "qhuff_tables.h"

namespace qhuff {

constexpr int kTile = 256;                 // strings per tile = threads per WG
constexpr int kEncInCap = 16 * 1024;       // staged input bytes per encode tile
constexpr int kDecInCap = 12 * 1024;       // staged input bytes per decode tile
constexpr int kSlot = 100;                 // LDS output slot per decode lane
                                           // (25 dwords: odd stride, no bank conflicts)

// ablation switches (timing experiments only; outputs are wrong when set)
constexpr uint32_t kDbgNoTicket = 1;       // tile = blockIdx.x
constexpr uint32_t kDbgNoLookback = 2;     // base = tile * 64 KiB
constexpr uint32_t kDbgNoStore = 4;        // skip output stores
constexpr uint32_t kDbgNoCodec = 8;        // skip the per-string codec loop

// look-back flag word: [63:62] state, [61:40] epoch, [39:0] inclusive or
// aggregate byte count
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 40) - 1;
constexpr uint32_t kEpochMask = (1u << 22) - 1;

struct DevTables
{
    uint32_t win[kWinSize];                // 16-byte aligned: copied as uint4
    uint2 enc[257];                        // {code, bits}
    uint16_t sorted[257];
};

struct LongParams
{
    LongLen l[kMaxLong];
    uint32_t n;
};

// ---------------------------------------------------------------------------
// small device helpers

__device__ __forceinline__ uint32_t
bswap32(uint32_t v)
{
    return __builtin_bswap32(v);
}

// bytes [p, p+4) of a little-endian dword stream whose dwords are lo, hi,
// starting at byte (p & 3) of lo
__device__ __forceinline__ uint32_t
align_bytes(uint32_t hi, uint32_t lo, uint32_t sh)
{
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// explicit address spaces: a generic pointer into LDS would compile to
// flat_load (global-memory latency) instead of ds_read
#define QH_LDS __attribute__((address_space(3)))
#define QH_GLB __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// uniform-per-launch source of aligned input dwords: LDS stage or global
struct LdsSrc
{
    const QH_LDS uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};

struct GlobalSrc
{
    const QH_GLB uint32_t *w;
    __device__ __forceinline__ uint32_t dw(uint32_t i) const { return w[i]; }
};

// workgroup exclusive scan of one uint32 per thread (256 threads, 4 waves)
__device__ __forceinline__ uint32_t
block_excl_scan(uint32_t v, uint32_t *s_wsum, uint32_t *total)
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
        s_wsum[wave] = x;
    __syncthreads();
    uint32_t w0 = s_wsum[0], w1 = s_wsum[1], w2 = s_wsum[2], w3 = s_wsum[3];
    uint32_t before = (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0)
                    + (wave > 2 ? w2 : 0);
    *total = w0 + w1 + w2 + w3;
    return before + x - v;
}

// Decoupled look-back (one wave): returns the exclusive byte prefix of
// `tile`, publishing the tile's inclusive value.  The aggregate was published
// by the caller already.
__device__ __forceinline__ uint64_t
look_back(unsigned long long *flags, uint32_t tile, uint64_t agg,
          uint32_t epoch)
{
    const int lane = threadIdx.x & 63;
    const uint64_t ep = (uint64_t) epoch << 40;
    uint64_t excl = 0;
    int64_t j = (int64_t) tile - 1;
    while (j >= 0)
    {
        int64_t idx = j - lane;
        uint64_t f = kFlagInc | ep;        // before tile 0: inclusive 0
        if (idx >= 0)
            f = __hip_atomic_load(&flags[idx], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        bool valid = ((f >> 40) & kEpochMask) == epoch && (f >> 62) != 0;
        bool inc = valid && (f >> 62) == 2;
        uint64_t incm = __ballot(inc);
        uint64_t invm = __ballot(!valid);
        // lanes [0, first inclusive] must all be valid
        uint64_t upto = incm ? ((incm & -incm) << 1) - 1 : ~0ull;
        if (invm & upto)
        {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t mine = (((upto >> lane) & 1) ? (f & kValMask) : 0);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1)
            mine += __shfl_xor(mine, d, 64);
        excl += mine;
        if (incm)
            break;
        j -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(&flags[tile], kFlagInc | ep | ((excl + agg) & kValMask),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// MSB-first bit packer writing big-endian bytes straight to global memory.
// Full aligned dwords are stored whole; the first and last dword of a string
// (shared with neighbouring strings) are stored byte by byte.
struct BitOut
{
    uint8_t *out;          // output base
    uint64_t acc;          // pending bits, left-aligned
    uint32_t nbits;        // bits in acc (includes the lead-in bytes)
    uint64_t wpos;         // byte position of the current (aligned) dword
    uint64_t lo, hi;       // bytes this string owns: [lo, hi)

    __device__ __forceinline__ void init(uint8_t *o, uint64_t start,
                                         uint64_t end)
    {
        out = o;
        lo = start;
        hi = end;
        wpos = start & ~3ull;
        nbits = 8u * (uint32_t) (start & 3);
        acc = 0;
    }

    __device__ __forceinline__ void store_word(uint32_t be)
    {
        if (wpos >= lo && wpos + 4 <= hi)
            *(uint32_t *) (out + wpos) = bswap32(be);
        else
        {
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                uint64_t p = wpos + k;
                if (p >= lo && p < hi)
                    out[p] = (uint8_t) (be >> (24 - 8 * k));
            }
        }
        wpos += 4;
    }

    __device__ __forceinline__ void put(uint32_t code, uint32_t len)
    {
        acc |= (uint64_t) code << (64 - nbits - len);
        nbits += len;
        if (nbits >= 32)
        {
            store_word((uint32_t) (acc >> 32));
            acc <<= 32;
            nbits -= 32;
        }
    }

    // pad to a byte boundary with the EOS prefix (ones), flush
    // (lsqpack.c:5171-5189)
    __device__ __forceinline__ void finish()
    {
        uint32_t pad = (8 - (nbits & 7)) & 7;
        if (pad)
            put((1u << pad) - 1, pad);
        while (nbits > 0)
        {
            store_word((uint32_t) (acc >> 32));
            acc <<= 32;
            nbits = nbits > 32 ? nbits - 32 : 0;
        }
    }
};

// ---------------------------------------------------------------------------
// encode

struct EncArgs
{
    const uint8_t *in;
    const uint32_t *in_off;
    uint8_t *out;
    uint32_t *out_off;
    const DevTables *tab;
    unsigned long long *flags;
    unsigned long long *ticket;
    unsigned long long ticket_base;
    uint32_t n;
    uint32_t epoch;
    uint32_t mode;            // 0 payload, 3/5/7 literal prefix bits
    uint32_t dbg;             // ablation switches (QHUFF_DEBUG), 0 in use
};

// number of bytes of an HPACK prefixed integer (lsqpack_val2len,
// lsqpack.c:767-783)
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

template <class Src>
__device__ __forceinline__ uint32_t
enc_bits(const Src &src, uint32_t rs, uint32_t re, const uint8_t *s_bits)
{
    uint32_t bits = 0;
    for (uint32_t d = rs >> 2; d * 4 < re; ++d)
    {
        uint32_t w = src.dw(d);
#pragma unroll
        for (int b = 0; b < 4; ++b)
        {
            uint32_t p = d * 4 + b;
            uint32_t l = s_bits[(w >> (8 * b)) & 0xff];
            bits += (p >= rs && p < re) ? l : 0;
        }
    }
    return bits;
}

template <class Src>
__device__ __forceinline__ void
enc_pack(const Src &src, uint32_t rs, uint32_t re, const uint2 *s_enc,
         BitOut &bo, bool raw)
{
    for (uint32_t d = rs >> 2; d * 4 < re; ++d)
    {
        uint32_t w = src.dw(d);
#pragma unroll
        for (int b = 0; b < 4; ++b)
        {
            uint32_t p = d * 4 + b;
            if (p >= rs && p < re)
            {
                uint32_t c = (w >> (8 * b)) & 0xff;
                if (raw)
                    bo.put(c, 8);
                else
                {
                    uint2 e = s_enc[c];
                    bo.put(e.x, e.y);
                }
            }
        }
    }
}

template <class Src>
__device__ __forceinline__ void
enc_tile_body(const EncArgs &a, const Src &src, uint32_t s, bool valid,
              uint32_t rs, uint32_t re, const uint2 *s_enc,
              const uint8_t *s_bits, uint32_t *s_wsum, uint64_t *s_base,
              uint32_t tile)
{
    const int tid = threadIdx.x;
    const uint32_t len = re - rs;
    uint32_t size = 0, plen = 0;
    bool huff = true;
    if (valid)
    {
        uint32_t hb = (a.dbg & kDbgNoCodec) ? len
                    : (enc_bits(src, rs, re, s_bits) + 7) >> 3;
        if (a.mode == 0)
            size = hb;
        else
        {
            huff = hb < len;                    // strict <, lsqpack.c:848
            plen = huff ? hb : len;
            size = int_len(plen, a.mode) + plen;
        }
    }
    uint32_t total;
    uint32_t excl = block_excl_scan(size, s_wsum, &total);

    if (tid == 0)
        __hip_atomic_store(&a.flags[tile],
                           kFlagAgg | ((uint64_t) a.epoch << 40) | total,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 64)
    {
        uint64_t base = (a.dbg & kDbgNoLookback) ? (uint64_t) tile << 16
                      : look_back(a.flags, tile, total, a.epoch);
        if (tid == 0)
            *s_base = base;
    }
    __syncthreads();
    const uint64_t base = *s_base;

    if (valid && !(a.dbg & kDbgNoStore))
    {
        a.out_off[s] = (uint32_t) (base + excl);
        if (s == a.n - 1)
            a.out_off[a.n] = (uint32_t) (base + excl + size);
        BitOut bo;
        bo.init(a.out, base + excl, base + excl + size);
        if (a.mode != 0)
        {
            // H bit + prefixed length (lsqpack.c:852-854, 863-864, 819-836)
            uint32_t P = a.mode, mask = (1u << P) - 1;
            uint32_t first = huff ? (1u << P) : 0;
            if (plen < mask)
                bo.put(first | plen, 8);
            else
            {
                bo.put(first | mask, 8);
                uint32_t v = plen - mask;
                while (v >= 128)
                {
                    bo.put(0x80 | (v & 0x7f), 8);
                    v >>= 7;
                }
                bo.put(v, 8);
            }
        }
        enc_pack(src, rs, re, s_enc, bo, !huff);
        bo.finish();
    }
}

__global__ __launch_bounds__(kTile) void
qhuff_encode_tile(EncArgs a)
{
    __shared__ uint2 s_enc[257];
    __shared__ uint8_t s_bits[256];
    __shared__ uint4 s_in[kEncInCap / 16 + 1];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_tile;

    const int tid = threadIdx.x;
    if (tid == 0)
        s_tile = (a.dbg & kDbgNoTicket) ? blockIdx.x
               : (uint32_t) (atomicAdd(a.ticket, 1ull) - a.ticket_base);
    s_enc[tid] = a.tab->enc[tid];
    s_bits[tid] = (uint8_t) a.tab->enc[tid].y;
    if (tid == 0)
        s_enc[256] = a.tab->enc[256];
    __syncthreads();

    const uint32_t tile = s_tile;
    const uint32_t s0 = tile * kTile;
    const uint32_t s = s0 + tid;
    const bool valid = s < a.n;
    const uint32_t last = min(s0 + kTile, a.n);
    const uint32_t A = a.in_off[s0], B = a.in_off[last];
    const uintptr_t pa = (uintptr_t) (a.in + A) & ~(uintptr_t) 15;
    const uintptr_t pb = ((uintptr_t) (a.in + B) + 15) & ~(uintptr_t) 15;
    uint32_t rs = 0, re = 0;
    if (valid)
    {
        rs = (uint32_t) ((uintptr_t) (a.in + a.in_off[s]) - pa);
        re = (uint32_t) ((uintptr_t) (a.in + a.in_off[s + 1]) - pa);
    }

    if (pb - pa <= (uintptr_t) kEncInCap)
    {
        const QH_GLB u32x4 *g = (const QH_GLB u32x4 *) pa;
        QH_LDS u32x4 *d4 = (QH_LDS u32x4 *) s_in;
        const uint32_t n16 = (uint32_t) ((pb - pa) >> 4);
        for (uint32_t i = tid; i < n16; i += kTile)
            d4[i] = g[i];
        __syncthreads();
        LdsSrc src{(const QH_LDS uint32_t *) s_in};
        enc_tile_body(a, src, s, valid, rs, re, s_enc, s_bits, s_wsum,
                      &s_base, tile);
    }
    else
    {
        GlobalSrc src{(const QH_GLB uint32_t *) pa};
        enc_tile_body(a, src, s, valid, rs, re, s_enc, s_bits, s_wsum,
                      &s_base, tile);
    }
}

// ---------------------------------------------------------------------------
// decode

struct DecArgs
{
    const uint8_t *in;
    const uint32_t *in_off;
    uint8_t *out;
    uint32_t *out_off;
    uint8_t *status;
    const DevTables *tab;
    unsigned long long *flags;
    unsigned long long *ticket;
    unsigned long long ticket_base;
    uint32_t n;
    uint32_t epoch;
    uint32_t dbg;
    LongParams lp;
};

// output sinks for the decoder
struct SlotSink                      // LDS slot, dword writes
{
    uint32_t *slot;
    uint64_t acc;
    uint32_t cnt, nw, cap_w;
    bool over;
    __device__ __forceinline__ void init(uint32_t *p, uint32_t cap_words)
    {
        slot = p;
        acc = 0;
        cnt = 0;
        nw = 0;
        cap_w = cap_words;
        over = false;
    }
    __device__ __forceinline__ void emit(uint32_t b)
    {
        acc |= (uint64_t) b << (8 * cnt);
        ++cnt;
    }
    __device__ __forceinline__ void settle()
    {
        if (cnt >= 4)
        {
            if (nw < cap_w)
                slot[nw] = (uint32_t) acc;
            else
                over = true;
            ++nw;
            acc >>= 32;
            cnt -= 4;
        }
    }
    __device__ __forceinline__ void finish()
    {
        if (cnt)
        {
            if (nw < cap_w)
                slot[nw] = (uint32_t) acc;
            else
                over = true;
        }
    }
    __device__ __forceinline__ uint32_t count() const { return nw * 4 + cnt; }
};

struct GlobalSink                    // direct byte stores (overflow path)
{
    uint8_t *dst;
    uint32_t n;
    __device__ __forceinline__ void emit(uint32_t b) { dst[n++] = (uint8_t) b; }
    __device__ __forceinline__ void settle() {}
    __device__ __forceinline__ void finish() {}
};

// 32 bits of the string starting at byte p (relative to the aligned source
// base) as a big-endian word; bytes at or past `re` read as 0xff (EOS
// padding, the way huff_decode_fast pads its last window, lsqpack.c:5364-5365)
template <class Src>
__device__ __forceinline__ uint32_t
fetch_be32(const Src &src, uint32_t p, uint32_t re)
{
    if (p >= re)
        return 0xffffffffu;
    uint32_t d = p >> 2, sh = p & 3;
    uint32_t lo = src.dw(d);
    uint32_t hi = ((d + 1) * 4 < re) ? src.dw(d + 1) : 0xffffffffu;
    uint32_t w = bswap32(align_bytes(hi, lo, sh));
    uint32_t valid = re - p;
    if (valid < 4)
        w |= 0xffffffffu >> (8 * valid);
    return w;
}

// Decode one complete string [rs, re) into `out`; returns true when the
// string is accepted (RFC 7541 5.2 / lsqpack.c:5362-5426 rule: no EOS,
// padding <= 7 bits, all ones).
template <class Src, class Sink>
__device__ __forceinline__ bool
dec_string(const Src &src, uint32_t rs, uint32_t re, const uint32_t *s_win,
           const uint16_t *s_sorted, const LongParams &lp, Sink &out)
{
    uint32_t p = rs;
    uint64_t buf = (uint64_t) fetch_be32(src, p, re) << 32;
    p += 4;
    buf |= fetch_be32(src, p, re);
    p += 4;
    uint32_t avail = 64;
    uint32_t left = 8 * (re - rs);           // real bits not yet consumed
    while (left > 0)
    {
        uint32_t e = s_win[buf >> (64 - kWinBits)];
        uint32_t ns = e >> 24;
        if (ns)
        {
            uint32_t l0 = (e >> 16) & 15, lt = (e >> 20) & 15;
            if (l0 > left)
                break;
            out.emit(e & 0xff);
            uint32_t c = l0;
            if (ns == 2 && lt <= left)
            {
                out.emit((e >> 8) & 0xff);
                c = lt;
            }
            out.settle();
            buf <<= c;
            avail -= c;
            left -= c;
        }
        else
        {
            // canonical decode of a code longer than kWinBits
            uint32_t w = (uint32_t) (buf >> 32);
            uint32_t L = 0, sym = 0;
            for (uint32_t i = 0; i < lp.n; ++i)
            {
                uint32_t v = w >> (32 - lp.l[i].len);
                uint32_t off = v - lp.l[i].first;
                if (L == 0 && off < lp.l[i].count)
                {
                    L = lp.l[i].len;
                    sym = s_sorted[lp.l[i].base + off];
                }
            }
            if (L > left)
                break;
            if (sym == 256)                  // EOS inside the string
                return false;
            out.emit(sym);
            out.settle();
            buf <<= L;
            avail -= L;
            left -= L;
        }
        if (avail < 32)
        {
            buf |= (uint64_t) fetch_be32(src, p, re) << (32 - avail);
            p += 4;
            avail += 32;
        }
    }
    out.finish();
    if (left >= 8)                            // padding longer than 7 bits
        return false;
    if (left)                                 // padding must be EOS prefix
    {
        uint64_t m = ~0ull << (64 - left);
        if ((buf & m) != m)
            return false;
    }
    return true;
}

template <class Src>
__device__ __forceinline__ void
dec_tile_body(const DecArgs &a, const Src &src, uint32_t s, bool valid,
              uint32_t rs, uint32_t re, const uint32_t *s_win,
              const uint16_t *s_sorted, uint32_t *s_slots, uint32_t *s_wsum,
              uint64_t *s_base, uint32_t tile)
{
    const int tid = threadIdx.x;
    uint32_t *slot = s_slots + tid * (kSlot / 4);
    uint32_t nout = 0;
    bool ok = true, over = false;
    if (valid && (a.dbg & kDbgNoCodec))
        nout = re - rs;
    else if (valid)
    {
        SlotSink sink;
        sink.init(slot, kSlot / 4);
        ok = dec_string(src, rs, re, s_win, s_sorted, a.lp, sink);
        over = sink.over;
        nout = ok ? sink.count() : 0;
    }
    uint32_t total;
    uint32_t excl = block_excl_scan(nout, s_wsum, &total);
    if (tid == 0)
        __hip_atomic_store(&a.flags[tile],
                           kFlagAgg | ((uint64_t) a.epoch << 40) | total,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid < 64)
    {
        uint64_t base = (a.dbg & kDbgNoLookback) ? (uint64_t) tile << 16
                      : look_back(a.flags, tile, total, a.epoch);
        if (tid == 0)
            *s_base = base;
    }
    __syncthreads();
    const uint64_t base = *s_base;
    if (!valid || (a.dbg & kDbgNoStore))
        return;
    a.out_off[s] = (uint32_t) (base + excl);
    a.status[s] = ok ? QHUFF_DEC_OK : QHUFF_DEC_ERROR;
    if (s == a.n - 1)
        a.out_off[a.n] = (uint32_t) (base + excl + nout);
    if (!ok || nout == 0)
        return;
    uint8_t *dst = a.out + base + excl;
    if (over)
    {
        // output did not fit the LDS slot: decode again straight to global
        GlobalSink gs{dst, 0};
        dec_string(src, rs, re, s_win, s_sorted, a.lp, gs);
        return;
    }
    // copy slot -> dst: head bytes, aligned dwords, tail bytes
    const uint8_t *sb = (const uint8_t *) slot;
    uint32_t head = (uint32_t) ((4 - ((uintptr_t) dst & 3)) & 3);
    if (head > nout)
        head = nout;
    for (uint32_t k = 0; k < head; ++k)
        dst[k] = sb[k];
    uint32_t nbody = (nout - head) >> 2;
    uint32_t *d4 = (uint32_t *) (dst + head);
    for (uint32_t k = 0; k < nbody; ++k)
    {
        uint32_t q = head + 4 * k;
        uint32_t lo = slot[q >> 2], hi = slot[(q >> 2) + 1];
        d4[k] = align_bytes(hi, lo, q & 3);
    }
    for (uint32_t k = head + 4 * nbody; k < nout; ++k)
        dst[k] = sb[k];
}

__global__ __launch_bounds__(kTile) void
qhuff_decode_tile(DecArgs a)
{
    __shared__ uint32_t s_win[kWinSize];
    __shared__ uint16_t s_sorted[257];
    __shared__ uint4 s_in[kDecInCap / 16 + 1];
    __shared__ uint32_t s_slots[kTile * kSlot / 4 + 1];
    __shared__ uint32_t s_wsum[4];
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_tile;

    const int tid = threadIdx.x;
    if (tid == 0)
        s_tile = (a.dbg & kDbgNoTicket) ? blockIdx.x
               : (uint32_t) (atomicAdd(a.ticket, 1ull) - a.ticket_base);
    {
        const uint4 *gw = (const uint4 *) a.tab->win;
        uint4 *sw = (uint4 *) s_win;
        for (int i = tid; i < kWinSize / 4; i += kTile)
            sw[i] = gw[i];
        s_sorted[tid] = a.tab->sorted[tid];
        if (tid == 0)
            s_sorted[256] = a.tab->sorted[256];
    }
    __syncthreads();

    const uint32_t tile = s_tile;
    const uint32_t s0 = tile * kTile;
    const uint32_t s = s0 + tid;
    const bool valid = s < a.n;
    const uint32_t last = min(s0 + kTile, a.n);
    const uint32_t A = a.in_off[s0], B = a.in_off[last];
    const uintptr_t pa = (uintptr_t) (a.in + A) & ~(uintptr_t) 15;
    const uintptr_t pb = ((uintptr_t) (a.in + B) + 15) & ~(uintptr_t) 15;
    uint32_t rs = 0, re = 0;
    if (valid)
    {
        rs = (uint32_t) ((uintptr_t) (a.in + a.in_off[s]) - pa);
        re = (uint32_t) ((uintptr_t) (a.in + a.in_off[s + 1]) - pa);
    }
    if (pb - pa <= (uintptr_t) kDecInCap)
    {
        const QH_GLB u32x4 *g = (const QH_GLB u32x4 *) pa;
        QH_LDS u32x4 *d4 = (QH_LDS u32x4 *) s_in;
        const uint32_t n16 = (uint32_t) ((pb - pa) >> 4);
        for (uint32_t i = tid; i < n16; i += kTile)
            d4[i] = g[i];
        __syncthreads();
        LdsSrc src{(const QH_LDS uint32_t *) s_in};
        dec_tile_body(a, src, s, valid, rs, re, s_win, s_sorted, s_slots,
                      s_wsum, &s_base, tile);
    }
    else
    {
        GlobalSrc src{(const QH_GLB uint32_t *) pa};
        dec_tile_body(a, src, s, valid, rs, re, s_win, s_sorted, s_slots,
                      s_wsum, &s_base, tile);
    }
}

}  // namespace qhuff

// ---------------------------------------------------------------------------
// host side: context, C-ABI

using namespace qhuff;

struct qhuff_ctx
{
    int device;
    hipStream_t own_stream;
    DevTables *tab;                      // device
    LongParams lp;
    unsigned long long *flags;           // device, cap_tiles entries
    unsigned long long *ticket;          // device, 1 entry
    uint64_t cap_tiles;
    unsigned long long ticket_base;
    uint32_t epoch;
    uint32_t dbg;                        // QHUFF_DEBUG ablation switches
    // host-path staging
    uint8_t *h_stage;                    // pinned
    size_t h_stage_cap;
    uint8_t *d_stage;
    size_t d_stage_cap;
    char err[256];
};

static int
fail(qhuff_ctx *c, hipError_t e, const char *what)
{
    if (c)
        snprintf(c->err, sizeof(c->err), "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? QHUFF_ENOMEM : QHUFF_EDEVICE;
}

#define HIPCHK(c, call)                                                      \
    do {                                                                     \
        hipError_t e_ = (call);                                              \
        if (e_ != hipSuccess)                                                \
            return fail((c), e_, #call);                                     \
    } while (0)

extern "C" int
qhuff_open(int device, qhuff_ctx **ctx_out)
{
    if (!ctx_out)
        return QHUFF_EINVAL;
    *ctx_out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return QHUFF_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return QHUFF_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return QHUFF_ENODEV;              // code objects are gfx950 only
    qhuff_ctx *c = new (std::nothrow) qhuff_ctx();
    if (!c)
        return QHUFF_ENOMEM;
    c->device = device;
    HIPCHK(c, hipSetDevice(device));
    HostTables *ht = new HostTables;
    build_tables(ht);
    DevTables dt;
    for (int i = 0; i < 257; ++i)
        dt.enc[i] = make_uint2(ht->code[i], ht->bits[i]);
    memcpy(dt.win, ht->win, sizeof(dt.win));
    memcpy(dt.sorted, ht->sorted, sizeof(dt.sorted));
    memset(&c->lp, 0, sizeof(c->lp));
    c->lp.n = ht->n_long;
    memcpy(c->lp.l, ht->longc, sizeof(LongLen) * ht->n_long);
    delete ht;
    int rc;
    hipError_t e = hipMalloc((void **) &c->tab, sizeof(DevTables));
    if (e != hipSuccess)
    {
        rc = fail(c, e, "hipMalloc tables");
        delete c;
        return rc;
    }
    e = hipMemcpy(c->tab, &dt, sizeof(dt), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMalloc((void **) &c->ticket, sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMemset(c->ticket, 0, sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess)
    {
        rc = fail(c, e, "context setup");
        qhuff_close(c);
        return rc;
    }
    c->epoch = 0;
    {
        const char *d = getenv("QHUFF_DEBUG");
        c->dbg = d ? (uint32_t) strtoul(d, nullptr, 0) : 0;
    }
    *ctx_out = c;
    return QHUFF_OK;
}

extern "C" void
qhuff_close(qhuff_ctx *c)
{
    if (!c)
        return;
    (void) hipSetDevice(c->device);
    if (c->own_stream)
        (void) hipStreamSynchronize(c->own_stream);
    (void) hipDeviceSynchronize();
    if (c->tab)
        (void) hipFree(c->tab);
    if (c->flags)
        (void) hipFree(c->flags);
    if (c->ticket)
        (void) hipFree(c->ticket);
    if (c->d_stage)
        (void) hipFree(c->d_stage);
    if (c->h_stage)
        (void) hipHostFree(c->h_stage);
    if (c->own_stream)
        (void) hipStreamDestroy(c->own_stream);
    delete c;
}

extern "C" const char *
qhuff_last_error(qhuff_ctx *c)
{
    return c ? c->err : "no context";
}

extern "C" uint64_t
qhuff_encode_bound(uint64_t in_bytes, uint32_t n, unsigned mode)
{
    // 30-bit longest code: ceil(30 * len / 8) per string; framing adds at
    // most 6 bytes of prefixed length (32-bit value) per literal
    uint64_t b = (in_bytes * 30 + 7) / 8 + n;
    if (mode)
        b += 6ull * n;
    return b + 16;
}

extern "C" uint64_t
qhuff_decode_bound(uint64_t in_bytes, uint32_t n)
{
    (void) n;
    return in_bytes * 8 / 5 + 16;
}

// make room for the look-back flags of `tiles` tiles and advance the epoch
static int
prepare_launch(qhuff_ctx *c, uint64_t tiles, hipStream_t st)
{
    if (tiles > c->cap_tiles)
    {
        if (c->flags)
        {
            HIPCHK(c, hipStreamSynchronize(st));
            HIPCHK(c, hipFree(c->flags));
            c->flags = nullptr;
        }
        uint64_t cap = tiles < 4096 ? 4096 : tiles;
        HIPCHK(c, hipMalloc((void **) &c->flags, cap * 8));
        HIPCHK(c, hipMemsetAsync(c->flags, 0, cap * 8, st));
        c->cap_tiles = cap;
    }
    c->epoch = (c->epoch + 1) & kEpochMask;
    if (c->epoch == 0)
    {
        // wrapped: stale flags could alias the new epoch
        HIPCHK(c, hipMemsetAsync(c->flags, 0, c->cap_tiles * 8, st));
        c->epoch = 1;
    }
    return QHUFF_OK;
}

extern "C" int
qhuff_encode_batch(qhuff_ctx *c, const uint8_t *in, const uint32_t *in_off,
                   uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off,
                   void *stream)
{
    if (!c || !in_off || !out_off || (n && (!in || !out)))
        return QHUFF_EINVAL;
    if (mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    hipStream_t st = (hipStream_t) stream;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0)
    {
        HIPCHK(c, hipMemsetAsync(out_off, 0, 4, st));
        return QHUFF_OK;
    }
    uint64_t tiles = (n + kTile - 1) / kTile;
    int rc = prepare_launch(c, tiles, st);
    if (rc)
        return rc;
    EncArgs a;
    a.in = in;
    a.in_off = in_off;
    a.out = out;
    a.out_off = out_off;
    a.tab = c->tab;
    a.flags = c->flags;
    a.ticket = c->ticket;
    a.ticket_base = c->ticket_base;
    a.n = n;
    a.epoch = c->epoch;
    a.mode = mode;
    a.dbg = c->dbg;
    hipLaunchKernelGGL(qhuff_encode_tile, dim3((uint32_t) tiles), dim3(kTile),
                       0, st, a);
    HIPCHK(c, hipGetLastError());
    c->ticket_base += tiles;
    return QHUFF_OK;
}

extern "C" int
qhuff_decode_batch(qhuff_ctx *c, const uint8_t *in, const uint32_t *in_off,
                   uint32_t n, uint8_t *out, uint32_t *out_off,
                   uint8_t *status, void *stream)
{
    if (!c || !in_off || !out_off || (n && (!in || !out || !status)))
        return QHUFF_EINVAL;
    hipStream_t st = (hipStream_t) stream;
    HIPCHK(c, hipSetDevice(c->device));
    if (n == 0)
    {
        HIPCHK(c, hipMemsetAsync(out_off, 0, 4, st));
        return QHUFF_OK;
    }
    uint64_t tiles = (n + kTile - 1) / kTile;
    int rc = prepare_launch(c, tiles, st);
    if (rc)
        return rc;
    DecArgs a;
    a.in = in;
    a.in_off = in_off;
    a.out = out;
    a.out_off = out_off;
    a.status = status;
    a.tab = c->tab;
    a.flags = c->flags;
    a.ticket = c->ticket;
    a.ticket_base = c->ticket_base;
    a.n = n;
    a.epoch = c->epoch;
    a.dbg = c->dbg;
    a.lp = c->lp;
    hipLaunchKernelGGL(qhuff_decode_tile, dim3((uint32_t) tiles), dim3(kTile),
                       0, st, a);
    HIPCHK(c, hipGetLastError());
    c->ticket_base += tiles;
    return QHUFF_OK;
}

// ---- host-memory path ------------------------------------------------------

static int
ensure_stage(qhuff_ctx *c, size_t bytes)
{
    if (bytes > c->h_stage_cap)
    {
        if (c->h_stage)
            (void) hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->h_stage_cap = 0;
        HIPCHK(c, hipHostMalloc((void **) &c->h_stage, bytes));
        c->h_stage_cap = bytes;
    }
    if (bytes > c->d_stage_cap)
    {
        if (c->d_stage)
            (void) hipFree(c->d_stage);
        c->d_stage = nullptr;
        c->d_stage_cap = 0;
        HIPCHK(c, hipMalloc((void **) &c->d_stage, bytes));
        c->d_stage_cap = bytes;
    }
    return QHUFF_OK;
}

static inline size_t
up16(size_t x)
{
    return (x + 15) & ~(size_t) 15;
}

// layout in both stages: [in bytes | in_off | out bytes | out_off | status]
static int
host_batch(qhuff_ctx *c, bool enc, const uint8_t *in, const uint32_t *in_off,
           uint32_t n, unsigned mode, uint8_t *out, uint32_t *out_off,
           uint8_t *status)
{
    if (!c || !in_off || !out_off || (n && (!in || !out)) || (!enc && n && !status))
        return QHUFF_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t a0 = in_off[0], in_bytes = (uint64_t) in_off[n] - a0;
    const uint64_t ob = enc ? qhuff_encode_bound(in_bytes, n, mode)
                            : qhuff_decode_bound(in_bytes, n);
    if (ob > 0xffffffffull)
        return QHUFF_ERANGE;
    size_t o_in = 0, o_off = up16(in_bytes), o_out = o_off + up16(4ull * (n + 1));
    size_t o_oo = o_out + up16(ob), o_st = o_oo + up16(4ull * (n + 1));
    size_t total = o_st + up16(n ? n : 1);
    int rc = ensure_stage(c, total);
    if (rc)
        return rc;
    hipStream_t st = c->own_stream;
    memcpy(c->h_stage + o_in, in + a0, in_bytes);
    uint32_t *hoff = (uint32_t *) (c->h_stage + o_off);
    for (uint32_t i = 0; i <= n; ++i)
        hoff[i] = in_off[i] - (uint32_t) a0;
    HIPCHK(c, hipMemcpyAsync(c->d_stage, c->h_stage, o_out,
                             hipMemcpyHostToDevice, st));
    if (enc)
        rc = qhuff_encode_batch(c, c->d_stage + o_in,
                                (const uint32_t *) (c->d_stage + o_off), n,
                                mode, c->d_stage + o_out,
                                (uint32_t *) (c->d_stage + o_oo), st);
    else
        rc = qhuff_decode_batch(c, c->d_stage + o_in,
                                (const uint32_t *) (c->d_stage + o_off), n,
                                c->d_stage + o_out,
                                (uint32_t *) (c->d_stage + o_oo),
                                c->d_stage + o_st, st);
    if (rc)
        return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_stage + o_oo, c->d_stage + o_oo,
                             4ull * (n + 1), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    memcpy(out_off, c->h_stage + o_oo, 4ull * (n + 1));
    uint64_t ot = out_off[n];
    size_t tail = enc ? 0 : up16(n);
    HIPCHK(c, hipMemcpyAsync(c->h_stage + o_out, c->d_stage + o_out, ot,
                             hipMemcpyDeviceToHost, st));
    if (!enc && n)
        HIPCHK(c, hipMemcpyAsync(c->h_stage + o_st, c->d_stage + o_st, tail,
                                 hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    memcpy(out, c->h_stage + o_out, ot);
    if (!enc && n)
        memcpy(status, c->h_stage + o_st, n);
    return QHUFF_OK;
}

extern "C" int
qhuff_encode_batch_host(qhuff_ctx *c, const uint8_t *in,
                        const uint32_t *in_off, uint32_t n, unsigned mode,
                        uint8_t *out, uint32_t *out_off)
{
    if (mode != 0 && mode != 3 && mode != 5 && mode != 7)
        return QHUFF_EINVAL;
    return host_batch(c, true, in, in_off, n, mode, out, out_off, nullptr);
}

extern "C" int
qhuff_decode_batch_host(qhuff_ctx *c, const uint8_t *in,
                        const uint32_t *in_off, uint32_t n, uint8_t *out,
                        uint32_t *out_off, uint8_t *status)
{
    return host_batch(c, false, in, in_off, n, 0, out, out_off, status);
}

// ---- per-string mirrors -----------------------------------------------------

extern "C" int
qhuff_enc_enc_str(qhuff_ctx *c, unsigned prefix_bits, unsigned char *dst,
                  size_t dst_len, const unsigned char *str, unsigned str_len)
{
    if (!c || !dst || (!str && str_len) || (prefix_bits != 3
            && prefix_bits != 5 && prefix_bits != 7))
        return -1;
    uint32_t off[2] = {0, str_len};
    uint64_t bound = qhuff_encode_bound(str_len, 1, prefix_bits);
    unsigned char *tmp = (unsigned char *) malloc(bound);
    unsigned char dummy = 0;
    uint32_t oo[2];
    if (!tmp)
        return -1;
    int rc = qhuff_encode_batch_host(c, str_len ? str : &dummy, off, 1,
                                     prefix_bits, tmp, oo);
    int r = -1;
    if (rc == QHUFF_OK && oo[1] <= dst_len)
    {
        // keep dst[0] bits above the H bit (lsqpack.c:852, 863)
        unsigned char keep = dst[0] & (unsigned char) ~((1u << (prefix_bits + 1)) - 1);
        memcpy(dst, tmp, oo[1]);
        dst[0] |= keep;
        r = (int) oo[1];
    }
    free(tmp);
    return r;
}

extern "C" unsigned
qhuff_enc_str_size(qhuff_ctx *c, const unsigned char *str, unsigned str_len)
{
    if (!c || (!str && str_len))
        return 0;
    uint32_t off[2] = {0, str_len};
    uint64_t bound = qhuff_encode_bound(str_len, 1, 0);
    unsigned char *tmp = (unsigned char *) malloc(bound);
    unsigned char dummy = 0;
    uint32_t oo[2] = {0, 0};
    if (!tmp)
        return 0;
    int rc = qhuff_encode_batch_host(c, str_len ? str : &dummy, off, 1, 0, tmp,
                                     oo);
    free(tmp);
    return rc == QHUFF_OK ? oo[1] : 0;
}

extern "C" struct qhuff_decode_retval
qhuff_huff_decode(qhuff_ctx *c, const unsigned char *src, int src_len,
                  unsigned char *dst, int dst_len)
{
    struct qhuff_decode_retval rv = {QHUFF_HUFF_DEC_ERROR, 0, 0};
    if (!c || src_len < 0 || dst_len < 0 || (!src && src_len))
        return rv;
    uint32_t off[2] = {0, (uint32_t) src_len};
    uint64_t bound = qhuff_decode_bound((uint64_t) src_len, 1);
    unsigned char *tmp = (unsigned char *) malloc(bound);
    unsigned char dummy = 0;
    uint32_t oo[2] = {0, 0};
    uint8_t status = QHUFF_DEC_ERROR;
    if (!tmp)
        return rv;
    int rc = qhuff_decode_batch_host(c, src_len ? src : &dummy, off, 1, tmp,
                                     oo, &status);
    if (rc == QHUFF_OK && status == QHUFF_DEC_OK)
    {
        if (oo[1] <= (uint32_t) dst_len)
        {
            memcpy(dst, tmp, oo[1]);
            rv.status = QHUFF_HUFF_DEC_OK;
            rv.n_dst = oo[1];
            rv.n_src = (unsigned) src_len;
        }
        else
            rv.status = QHUFF_HUFF_DEC_END_DST;
    }
    free(tmp);
    return rv;
}

// ---- host helpers --------------------------------------------------------------

extern "C" int
qhuff_shard_cuts(const uint32_t *in_off, uint32_t n, uint32_t g,
                 uint32_t *cuts)
{
    if (!in_off || !cuts || g == 0)
        return QHUFF_EINVAL;
    const uint64_t a = in_off[0], tot = (uint64_t) in_off[n] - a;
    cuts[0] = 0;
    uint32_t i = 0;
    for (uint32_t k = 1; k < g; ++k)
    {
        uint64_t target = a + tot * k / g;
        // first string index whose start offset reaches the target
        uint32_t lo = i, hi = n;
        while (lo < hi)
        {
            uint32_t mid = lo + (hi - lo) / 2;
            if (in_off[mid] < target)
                lo = mid + 1;
            else
                hi = mid;
        }
        i = lo;
        cuts[k] = i;
    }
    cuts[g] = n;
    return QHUFF_OK;
}

extern "C" uint64_t
qhuff_synth_batch(uint64_t seed, uint32_t n, uint32_t min_len,
                  uint32_t max_len, const uint8_t *alphabet,
                  uint32_t alphabet_len, uint8_t *data, uint32_t *in_off)
{
    uint64_t x = seed ? seed : 0x9E3779B97F4A7C15ull;
    uint64_t pos = 0;
    const uint32_t span = max_len - min_len + 1;
    for (uint32_t i = 0; i < n; ++i)
    {
        in_off[i] = (uint32_t) pos;
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        uint32_t len = min_len + (uint32_t) (x % span);
        for (uint32_t k = 0; k < len; ++k)
        {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            data[pos++] = alphabet[x % alphabet_len];
        }
    }
    in_off[n] = (uint32_t) pos;
    return pos;
}
