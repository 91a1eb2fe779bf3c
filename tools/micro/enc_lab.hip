// Encode phase lab: the real kernel's dense pass, sizing and emit
// (qhuff_encode.hip) run R times on a tile staged once in each wave's LDS
// region, at 1 and 12 waves per CU.  Prints cycles per tile per wave for
// each phase.  Build:
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//       [-DQH_ENC_WORDS_ROWS=G] enc_lab.hip ../../ls-qpack_amd/csrc/qhuff_tables.cpp
// Odd repetitions time the word-parallel emit below, even ones the kernel's;
// both outputs are compared word for word once per wave first.
#include "../../ls-qpack_amd/csrc/qhuff_encode.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

using namespace qhuff;

// VERDICT r04 item 5's word-parallel emit, built here to be measured against
// the kernel's string-per-lane emit (EncPolicyT::emit); not in the kernels
// (2.8-3.0x the emit's cycles at 1, 4 and 12 waves/CU)
namespace qhuff {
#ifndef QH_ENC_WORDS_ROWS                   // emit_words: rows per group
#define QH_ENC_WORDS_ROWS 4
#endif

// inclusive maximum scan over the wave (VALU only, as wave_incl_scan)
__device__ __forceinline__ uint32_t
wave_incl_max(uint32_t v)
{
    uint32_t x = v;
    x = max(x, dpp0<0x111, 0xf>(x));
    x = max(x, dpp0<0x112, 0xf>(x));
    x = max(x, dpp0<0x114, 0xf>(x));
    x = max(x, dpp0<0x118, 0xf>(x));
    x = max(x, dpp0<0x142, 0xa>(x));
    x = max(x, dpp0<0x143, 0xc>(x));
    return x;
}

// Word-parallel emit of a dense mode-0 tile (every string Huffman-coded,
// from the dense stream): lane l writes output words l, l + 64, ... whole,
// whatever strings they hold, so the wave no longer runs to its longest
// string.  Each word finds the string holding its first byte by a running
// maximum over marks (string j + 1 at the first word starting at or after
// its first byte), then takes that string's bits -- a 32-bit window of the
// dense stream, its EOS-prefix padding -- and the following strings' while
// they start inside the word.  The marks overwrite the input stage and the
// strings' ranges the chunk offsets (both dead once the codec has run).
__device__ __forceinline__ void
emit_words(QH_LDS EncWave *wv, uint32_t cnt, uint32_t excl, uint32_t sz,
           uint32_t ds, uint32_t bits, uint32_t total)
{
    const uint32_t lane = lane_id();
    QH_LDS uint32_t *mk = wv->in;
    QH_LDS u32x2 *pr = (QH_LDS u32x2 *) wv->s0;
    const uint32_t nw = (total + 3) >> 2;
    for (uint32_t i = lane; i < (nw + 3) >> 2; i += 64)
        ((QH_LDS u32x4 *) mk)[i] = (u32x4){0, 0, 0, 0};
    pr[lane] = (u32x2){excl | (ds << 12), bits | ((excl + sz) << 16)};
    wave_sync();
    const uint32_t c = (excl + 3) >> 2;
    if ((lane < cnt) & (c < nw))
        __hip_atomic_fetch_max(&mk[c], lane + 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    wave_sync();
    uint32_t carry = 0;
#if QH_ENC_WORDS_ROWS > 1
    // rows in groups, every LDS read of a step issued for the whole group
    // before its results are used: the marks; the ranges of the word's first
    // string and the next; both strings' dense windows (the second only
    // where the first ends inside the word); a loop for further strings
    constexpr int G = QH_ENC_WORDS_ROWS;
    const uint32_t jl = cnt - 1;
    for (uint32_t w0 = 0; w0 < nw; w0 += 64 * G)
    {
        uint32_t m[G], j[G], v[G];
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            const uint32_t w = w0 + 64 * k + lane;
            m[k] = w < nw ? mk[w] : 0u;
        }
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            m[k] = wave_incl_max(m[k]);
            j[k] = min(max(m[k], carry) - 1, jl);
            carry = max(carry, read_lane(m[k], 63));
        }
        u32x2 q[G], r[G];
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            q[k] = pr[j[k]];
            r[k] = pr[min(j[k] + 1, jl)];
        }
        uint32_t a[G], b[G], c2[G], d2[G], s[G], t[G];
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            const uint32_t p = 32 * (w0 + 64 * k + lane);
            const uint32_t sb = 8 * (q[k].x & 0xfffu);
            s[k] = (q[k].x >> 12) + (p > sb ? p - sb : 0u);
            const uint32_t d = min(s[k] >> 5, (uint32_t) kDenseWords - 2);
            a[k] = wv->dense[d];
            b[k] = wv->dense[d + 1];
            // (read whether or not it is needed: a branch here costs a
            // full wait for the group's reads)
            t[k] = r[k].x >> 12;
            const uint32_t e = min(t[k] >> 5, (uint32_t) kDenseWords - 2);
            c2[k] = wv->dense[e];
            d2[k] = wv->dense[e + 1];
        }
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            const uint32_t w = w0 + 64 * k + lane;
            const uint32_t p = 32 * w, pe = p + 32;
            // a string's bits within the word: its dense window from bit
            // `src` (the window's first bit `lead` bits into the word), its
            // padding ones to its end
            auto seg = [&](uint32_t x, uint32_t lead, uint32_t pb, uint32_t eb) {
                x = lead ? x >> lead : x;
                const uint32_t q1 = pb > p ? min(pb - p, 32u) : 0u;
                const uint32_t q2 = eb > p ? min(eb - p, 32u) : 0u;
                const uint32_t mp = q1 ? 0xffffffffu << (32 - q1) : 0u;
                const uint32_t ms = q2 ? 0xffffffffu << (32 - q2) : 0u;
                return (x & mp) | (ms & ~mp);
            };
            auto win = [](uint32_t x, uint32_t y, uint32_t src) {
                return (src & 31) ? __builtin_amdgcn_alignbit(x, y, 32 - (src & 31))
                                  : x;
            };
            uint32_t eb = 8 * (q[k].y >> 16);
            v[k] = seg(win(a[k], b[k], s[k]), 0u,
                       8 * (q[k].x & 0xfffu) + (q[k].y & 0xffffu), eb);
            uint32_t jj = j[k];
            if ((eb < pe) & (jj < jl))
            {
                ++jj;
                const uint32_t sb = 8 * (r[k].x & 0xfffu);
                eb = 8 * (r[k].y >> 16);
                v[k] |= seg(win(c2[k], d2[k], t[k]), sb - p,
                            sb + (r[k].y & 0xffffu), eb);
                // (rare) strings of under 4 bytes inside the word
                while ((eb < pe) & (jj < jl) & (w < nw))
                {
                    ++jj;
                    const u32x2 u = pr[jj];
                    const uint32_t sb3 = 8 * (u.x & 0xfffu), ss = u.x >> 12;
                    eb = 8 * (u.y >> 16);
                    const uint32_t e = min(ss >> 5, (uint32_t) kDenseWords - 2);
                    v[k] |= seg(win(wv->dense[e], wv->dense[e + 1], ss), sb3 - p,
                                sb3 + (u.y & 0xffffu), eb);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < G; ++k)
        {
            const uint32_t w = w0 + 64 * k + lane;
            if (w < nw)
                wv->out[w] = bswap32(v[k]);
        }
    }
    return;
#endif
    for (uint32_t w0 = 0; w0 < nw; w0 += 64)
    {
        const uint32_t w = w0 + lane;
        const uint32_t m = wave_incl_max(w < nw ? mk[w] : 0u);
        uint32_t j = max(m, carry) - 1;
        carry = max(carry, read_lane(m, 63));
        if (w >= nw)
            continue;
        const uint32_t p = 32 * w, pe = p + 32;
        uint32_t v = 0;
        for (;;)
        {
            const u32x2 q = pr[j];
            const uint32_t sb = 8 * (q.x & 0xfffu), s0 = q.x >> 12;
            const uint32_t pb = sb + (q.y & 0xffffu), eb = 8 * (q.y >> 16);
            const uint32_t lead = sb > p ? sb - p : 0u;   // string starts inside
            const uint32_t s = s0 + (p > sb ? p - sb : 0u);
            const uint32_t d = min(s >> 5, (uint32_t) kDenseWords - 2);
            const uint32_t a = wv->dense[d], b = wv->dense[d + 1];
            uint32_t x = (s & 31) ? __builtin_amdgcn_alignbit(a, b, 32 - (s & 31))
                                  : a;
            x = lead ? x >> lead : x;
            const uint32_t q1 = pb > p ? min(pb - p, 32u) : 0u;
            const uint32_t q2 = eb > p ? min(eb - p, 32u) : 0u;
            const uint32_t mp = q1 ? 0xffffffffu << (32 - q1) : 0u;
            const uint32_t ms = q2 ? 0xffffffffu << (32 - q2) : 0u;
            v |= (x & mp) | (ms & ~mp);
            if ((eb >= pe) | (j + 1 >= cnt))
                break;
            ++j;
        }
        wv->out[w] = bswap32(v);
    }
}

} // namespace qhuff

struct MbOut { unsigned long long c_dense, c_size, c_emit, c_words, sum, bad; };

template <int W>
__global__ __launch_bounds__(64 * W) void
enc_lab(EncArgs a, int reps, MbOut *res)
{
    __shared__ EncSmem smem;
    QH_LDS EncSmem *sm = (QH_LDS EncSmem *) &smem;
    const int tid = threadIdx.x;
    for (int i = tid; i < 257; i += 64 * W)  // (the kernel's 768 threads: one each)
        enc_tables_load(sm, a.enc, i);
    __syncthreads();
    QH_LDS EncWave *wv = &sm->w[tid >> 6];
    const uint32_t gid = blockIdx.x * W + (tid >> 6), lane = lane_id();
    const uint32_t t = gid % a.c.n_tiles;
    TileOffs to;
    to.load((const QH_GLB uint32_t *) a.in_off, (uint64_t) t * kWT, kWT);
    const Span sp = tile_span(a.in, to.first(), to.last(), kStageCap);
    Chunks<kChunks> ch;
    ch.load(sp);
    EncPolicyT<EncSmem, false> pol;
    pol.in = a.in;
    pol.mode = a.mode;
    pol.sm = sm;
    pol.wv = wv;
    pol.dense = false;
    pol.stage_in(ch, sp, to);
    wave_sync();
    unsigned long long cd = 0, cs = 0, ce = 0, cw = 0, sum = 0, bad = 0;
    // parity of the word-parallel emit against the kernel's, once
    {
        pol.prepare(sp);
        wave_sync();
        uint32_t sz, st;
        pol.codec(to, kWT, sp, &sz, &st);
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t total = read_lane(incl, 63);
        wave_sync();
        pol.emit(incl - sz, sz, total);
        wave_sync();
        const uint32_t nw = (total + 3) >> 2;
        uint32_t ref[12];
#pragma unroll
        for (int r = 0; r < 12; ++r)
            ref[r] = 64 * r + lane < nw ? wv->out[64 * r + lane] : 0u;
        wave_sync();
        // the dense stream against the bit packer on the staged input
        {
            QH_LDS u32x4 *o4 = (QH_LDS u32x4 *) wv->out;
            for (uint32_t i = lane; i < (total + 15) / 16 + 1; i += 64)
                o4[i] = (u32x4){0, 0, 0, 0};
            wave_sync();
            if (sz)
                emit_bits(wv->in, pol.rs, pol.re, pol.mode, pol.z.huff, pol.z.plen,
                          sm->enc, wv->out, incl - sz);
            wave_sync();
#pragma unroll
            for (int r = 0; r < 12; ++r)
                bad += 64 * r + lane < nw && wv->out[64 * r + lane] != ref[r];
            wave_sync();
        }
        if (pol.dense)
            emit_words(wv, kWT, incl - sz, sz, pol.ds, pol.bits, total);
        wave_sync();
#pragma unroll
        for (int r = 0; r < 12; ++r)
            bad += 64 * r + lane < nw && wv->out[64 * r + lane] != ref[r];
        bad += pol.dense ? 0 : 1000000;
        pol.stage_in(ch, sp, to);
        wave_sync();
    }
    for (int r = 0; r < reps; ++r)
    {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        pol.prepare(sp);                     // the dense pass
        wave_sync();
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        uint32_t sz, st;
        pol.codec(to, kWT, sp, &sz, &st);
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t total = read_lane(incl, 63);
        wave_sync();
        const uint64_t t2 = __builtin_amdgcn_s_memtime();
        if (r & 1)
            emit_words(wv, kWT, incl - sz, sz, pol.ds, pol.bits, total);
        else
            pol.emit(incl - sz, sz, total);
        wave_sync();
        sum += wv->out[lane] + total + (pol.dense ? 1 : 0);
        const uint64_t t3 = __builtin_amdgcn_s_memtime();
        cd += t1 - t0;
        cs += t2 - t1;
        (r & 1 ? cw : ce) += t3 - t2;
        if (r & 1)                           // the marks overwrote the stage
        {
            pol.stage_in(ch, sp, to);
            wave_sync();
        }
    }
    if (lane == 0)
    {
        res[gid].c_dense = cd / reps;
        res[gid].c_size = cs / reps;
        res[gid].c_emit = ce / (reps / 2);
        res[gid].c_words = cw / (reps / 2);
        res[gid].sum = sum;
    }
    const uint64_t bm = __builtin_amdgcn_ballot_w64(bad != 0);
    if (lane == 0)
        res[gid].bad = bm ? 1 : 0;
}

static void synth(uint32_t n, std::vector<uint8_t> &data, std::vector<uint32_t> &off)
{
    const char *alpha = "abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, ";
    const uint32_t al = 45;
    uint64_t x = 0x9E3779B97F4A7C15ull;
    off.resize(n + 1);
    data.clear();
    for (uint32_t i = 0; i < n; ++i)
    {
        off[i] = (uint32_t) data.size();
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        uint32_t len = 8 + (uint32_t) (x % 57);
        for (uint32_t k = 0; k < len; ++k)
        {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            data.push_back((uint8_t) alpha[x % al]);
        }
    }
    off[n] = (uint32_t) data.size();
}

template <int W>
static void run(const EncArgs &a, int reps)
{
    const int blocks = 256, nw = blocks * W;
    MbOut *d;
    (void) hipMalloc(&d, sizeof(MbOut) * nw);
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((enc_lab<W>), dim3(blocks), dim3(64 * W), 0, 0, a,
                           reps, d);
    (void) hipDeviceSynchronize();
    std::vector<MbOut> h(nw);
    (void) hipMemcpy(h.data(), d, sizeof(MbOut) * nw, hipMemcpyDeviceToHost);
    double x = 0, y = 0, z = 0, u = 0;
    unsigned long long bad = 0;
    for (auto &o : h)
    {
        x += o.c_dense; y += o.c_size; z += o.c_emit; u += o.c_words;
        bad += o.bad;
    }
    printf("%2d waves/CU: dense %6.0f  sizing+scan %6.0f  emit %6.0f  "
           "word emit %6.0f  cycles/tile/wave  (waves differing: %llu)\n",
           W, x / nw, y / nw, z / nw, u / nw, bad);
    (void) hipFree(d);
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    const uint32_t n = 1 << 20;
    std::vector<uint8_t> data;
    std::vector<uint32_t> off;
    synth(n, data, off);
    HostTables ht;
    build_tables(&ht);
    uint8_t *d_in;
    uint32_t *d_off;
    uint2 *d_enc;
    (void) hipMalloc(&d_in, data.size() + 64);
    (void) hipMalloc(&d_off, 4 * (n + 1));
    (void) hipMalloc(&d_enc, 8 * 257);
    (void) hipMemcpy(d_in, data.data(), data.size(), hipMemcpyHostToDevice);
    (void) hipMemcpy(d_off, off.data(), 4 * (n + 1), hipMemcpyHostToDevice);
    std::vector<uint2> enc(257);
    for (int i = 0; i < 257; ++i) enc[i] = make_uint2(ht.code[i], ht.bits[i]);
    (void) hipMemcpy(d_enc, enc.data(), 8 * 257, hipMemcpyHostToDevice);
    const int reps = argc > 1 ? atoi(argv[1]) : 32;
    EncArgs a = {};
    a.in = d_in; a.in_off = d_off; a.enc = d_enc; a.n = n; a.mode = 0;
    a.c.n_tiles = n / 64;
    run<1>(a, reps);
    run<4>(a, reps);
    run<12>(a, reps);
    return 0;
}
