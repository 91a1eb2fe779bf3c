// qhuff_hash.hip -- batched XXH32 of header names and values (gfx950).
//
// Reference: every header the encoder takes
// and every header the decoder emits is hashed twice with XXH32
// (deps/xxhash/xxhash.c, 32-bit variant):
//
//   name_hash    = XXH32(name,  name_len,  LSQPACK_XXH_SEED)  lsqpack.c:1681,
//                                                             3268-3269
//   nameval_hash = XXH32(value, value_len, name_hash)         lsqpack.c:1685,
//                                                             3308-3309
//
// (LSQPACK_XXH_SEED = 39378473, lsqpack.c:623).  The hashes index the static
// table (name2id_plus_one / nameval2id_plus_one, lsqpack.c:629-753) and the
// dynamic table.  Like the Huffman kernels this is per-string byte work:
// one header per lane, one 64-header tile per wave, the tile's contiguous
// name/value bytes staged into the wave's LDS region with coalesced 16-byte
// loads, then each lane walks its own bytes out of LDS (four 32-bit
// accumulators over 16-byte stripes, then 4-byte and 1-byte tails).  The
// outputs are fixed-size (two u32 per header), so no scan or look-back is
// needed; waves are persistent (grid = what is resident) and prefetch the
// next tile's bytes while hashing the current one.  HBM-bound: a header
// costs its name + value bytes + 8 B of offsets + 8 B of hashes.
#include "qhuff_kernels.h"

#include <hip/hip_ext.h>

namespace qhuff {

constexpr int kHashWaves = 8;                      // waves per workgroup
constexpr int kHashNch = 6;                        // 16-byte chunks per lane
constexpr uint32_t kHashCap = 64 * kHashNch * 16;  // staged bytes per wave

constexpr uint32_t kP1 = 2654435761u, kP2 = 2246822519u, kP3 = 3266489917u,
                   kP4 = 668265263u, kP5 = 374761393u;

__device__ __forceinline__ uint32_t
rotl32(uint32_t x, uint32_t r)
{
    return __builtin_amdgcn_alignbit(x, x, 32 - r);
}

__device__ __forceinline__ uint32_t
xxh_round(uint32_t acc, uint32_t w)
{
    return rotl32(acc + w * kP2, 13) * kP1;
}

// bytes staged in LDS; byte index i = global address - 16-aligned span base
struct HashLds
{
    const QH_LDS uint32_t *s;
    __device__ __forceinline__ uint32_t word(uint32_t i) const
    {
        const uint32_t q = i >> 2;
        return align_bytes(s[q + 1], s[q], i & 3);
    }
    __device__ __forceinline__ void stripe(uint32_t i, uint32_t w[4]) const
    {
        const uint32_t q = i >> 2, sh = i & 3;
        const uint32_t d0 = s[q], d1 = s[q + 1], d2 = s[q + 2], d3 = s[q + 3],
                       d4 = s[q + 4];
        w[0] = align_bytes(d1, d0, sh);
        w[1] = align_bytes(d2, d1, sh);
        w[2] = align_bytes(d3, d2, sh);
        w[3] = align_bytes(d4, d3, sh);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t i) const
    {
        return ((const QH_LDS uint8_t *) s)[i];
    }
};

// bytes read straight from global (tiles too large for the stage): byte
// loads only, so nothing outside the string is touched
struct HashGlb
{
    const QH_GLB uint8_t *p;
    __device__ __forceinline__ uint32_t byte(uint32_t i) const { return p[i]; }
    __device__ __forceinline__ uint32_t word(uint32_t i) const
    {
        return p[i] | (p[i + 1] << 8) | (p[i + 2] << 16)
             | ((uint32_t) p[i + 3] << 24);
    }
    __device__ __forceinline__ void stripe(uint32_t i, uint32_t w[4]) const
    {
        w[0] = word(i);
        w[1] = word(i + 4);
        w[2] = word(i + 8);
        w[3] = word(i + 12);
    }
};

// XXH32 of bytes [a, a + len) (xxhash.c XXH32 / XXH32_endian_align):
// 16-byte stripes into four lanes, merge, + len, 4-byte then 1-byte tail,
// avalanche
template <class R>
__device__ __forceinline__ uint32_t
xxh32(const R &r, uint32_t a, uint32_t len, uint32_t seed)
{
    uint32_t p = a;
    const uint32_t end = a + len;
    uint32_t h;
    if (len >= 16)
    {
        uint32_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed,
                 v4 = seed - kP1;
        const uint32_t limit = end - 16;
        do
        {
            uint32_t w[4];
            r.stripe(p, w);
            v1 = xxh_round(v1, w[0]);
            v2 = xxh_round(v2, w[1]);
            v3 = xxh_round(v3, w[2]);
            v4 = xxh_round(v4, w[3]);
            p += 16;
        } while (p <= limit);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    }
    else
        h = seed + kP5;
    h += len;
    while (p + 4 <= end)
    {
        h += r.word(p) * kP3;
        h = rotl32(h, 17) * kP4;
        p += 4;
    }
    while (p < end)
    {
        h += r.byte(p) * kP5;
        h = rotl32(h, 11) * kP1;
        ++p;
    }
    h ^= h >> 15;
    h *= kP2;
    h ^= h >> 13;
    h *= kP3;
    h ^= h >> 16;
    return h;
}

struct HashWave
{
    alignas(16) uint32_t s[kHashCap / 4 + 8];      // + slack for stripe reads
};

template <class R>
__device__ __forceinline__ void
hash_lane(const R &r, bool pairs, uint32_t a, uint32_t m, uint32_t b,
          uint32_t seed, uint32_t *h1, uint32_t *h2)
{
    if (pairs)
    {
        *h1 = xxh32(r, a, m - a, seed);
        *h2 = xxh32(r, m, b - m, *h1);
    }
    else
        *h1 = xxh32(r, a, b - a, seed);
}

// a tile's offsets: lane l holds header/string l's start, name end (pairs)
// and end; every lane loads (clamped index), so the count is fixed
struct HashOffs
{
    uint32_t a, m, b, cnt;

    __device__ __forceinline__ void load(const QH_GLB uint32_t *off,
                                         uint64_t t, uint64_t n, bool pairs)
    {
        const uint64_t s0 = t * kWT;
        cnt = (uint32_t) min((uint64_t) kWT, n - s0);
        const uint32_t k = pairs ? 2 : 1;
        const uint32_t li = lane_id() < cnt ? lane_id() : cnt - 1;
        const QH_GLB uint32_t *o = off + s0 * k + k * li;
        a = o[0];
        m = o[1];
        b = pairs ? o[2] : m;
    }
    __device__ __forceinline__ uint32_t first() const { return read_lane(a, 0); }
    __device__ __forceinline__ uint32_t last() const
    {
        return read_lane(b, cnt - 1);
    }
};

// Persistent waves, software-pipelined like the codec kernels: while tile t
// is hashed out of LDS, the bytes of tile t + W and the offsets of tile
// t + 2W are already in flight (W = waves in the grid).
__global__ __launch_bounds__(64 * kHashWaves) void
qhuff_hash_kernel(HashArgs a)
{
    __shared__ HashWave sm[kHashWaves];
    const uint32_t lane = lane_id();
    const uint32_t wv = threadIdx.x >> 6;
    const uint64_t nt = (a.n + kWT - 1) / kWT;
    const uint64_t W = (uint64_t) gridDim.x * kHashWaves;
    uint64_t t = (uint64_t) blockIdx.x * kHashWaves + wv;
    if (t >= nt)
        return;
    const bool pairs = a.pairs != 0;
    const QH_GLB uint32_t *off = glb(a.off);
    auto clamp = [&](uint64_t x) { return x < nt ? x : nt - 1; };
    QH_LDS uint32_t *s = (QH_LDS uint32_t *) sm[wv].s;

    HashOffs o_cur, o_nxt, o_nn;
    o_cur.load(off, t, a.n, pairs);
    Span sp_cur = tile_span(a.in, o_cur.first(), o_cur.last(), kHashCap);
    Chunks<kHashNch> ch;
    ch.load(sp_cur);
    o_nxt.load(off, clamp(t + W), a.n, pairs);
    for (;;)
    {
        __builtin_amdgcn_s_waitcnt(0x0f70);           // vmcnt(0)
        if (sp_cur.staged)
            ch.store<false>((QH_LDS u32x4 *) s, sp_cur.n16);
        wave_sync();
        const Span sp_nxt = tile_span(a.in, o_nxt.first(), o_nxt.last(),
                                      kHashCap);
        if (t + W < nt)
            ch.load(sp_nxt);
        o_nn.load(off, clamp(t + 2 * W), a.n, pairs);

        uint32_t h1 = 0, h2 = 0;
        const uint32_t first = o_cur.first();
        if (sp_cur.staged)
        {
            // byte index of input offset x in the stage: x - first + skew
            const uint32_t skew = (uint32_t) ((uintptr_t) (a.in + first)
                                              - sp_cur.pa);
            const HashLds r{s};
            hash_lane(r, pairs, o_cur.a - first + skew, o_cur.m - first + skew,
                      o_cur.b - first + skew, a.seed, &h1, &h2);
        }
        else
        {
            const HashGlb r{glb(a.in)};
            hash_lane(r, pairs, o_cur.a, o_cur.m, o_cur.b, a.seed, &h1, &h2);
        }
        const uint64_t s0 = t * kWT;
        if (lane < o_cur.cnt)
        {
            glb(a.h1)[s0 + lane] = h1;
            if (pairs)
                glb(a.h2)[s0 + lane] = h2;
        }
        wave_sync();
        t += W;
        if (t >= nt)
            break;
        o_cur = o_nxt;
        o_nxt = o_nn;
        sp_cur = sp_nxt;
    }
}

hipError_t
launch_hash(const HashArgs &a, uint32_t max_grid, hipStream_t st,
            hipEvent_t ev0, hipEvent_t ev1)
{
    const uint64_t tiles = (a.n + kWT - 1) / kWT;
    const uint64_t need = (tiles + kHashWaves - 1) / kHashWaves;
    const uint32_t grid = (uint32_t) (need < max_grid ? need : max_grid);
    if (ev0)
        hipExtLaunchKernelGGL(qhuff_hash_kernel, dim3(grid),
                              dim3(64 * kHashWaves), 0, st, ev0, ev1, 0, a);
    else
        hipLaunchKernelGGL(qhuff_hash_kernel, dim3(grid), dim3(64 * kHashWaves),
                           0, st, a);
    return hipGetLastError();
}

// Shard stitching (qhuff_*_batch_multi): off[i] += add for i in [0, n],
// four offsets per lane with 16-byte accesses where the array allows
// (a grid-stride loop: every wave exits when its range is done).
__global__ __launch_bounds__(256) void
qhuff_rebase_kernel(uint32_t *off, uint64_t n, uint32_t add)
{
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    const uint64_t head = (4 - (((uintptr_t) off >> 2) & 3)) & 3;   // to 16 B
    const uint64_t h = head < n ? head : n;
    const uint64_t t = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t < h)
        off[t] += add;
    U4 *v = (U4 *) (off + h);
    const uint64_t nv = (n - h) / 4;
    for (uint64_t i = t; i < nv; i += stride)
    {
        u32x4 x = v[i].v;
        x.x += add;
        x.y += add;
        x.z += add;
        x.w += add;
        v[i].v = x;
    }
    for (uint64_t i = h + 4 * nv + t; i < n; i += stride)
        off[i] += add;
}

hipError_t
launch_rebase(uint32_t *off, uint64_t n, uint32_t add, hipStream_t st)
{
    if (n == 0 || add == 0)
        return hipSuccess;
    const uint64_t need = (n / 4 + 255) / 256 + 1;
    const uint32_t grid = (uint32_t) (need < 2048 ? need : 2048);
    hipLaunchKernelGGL(qhuff_rebase_kernel, dim3(grid), dim3(256), 0, st, off,
                       n, add);
    return hipGetLastError();
}

int
hash_waves_per_block()
{
    return kHashWaves;
}

hipError_t
hash_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_hash_kernel),
        64 * kHashWaves, 0);
}

}  // namespace qhuff
