// Codec microbenchmark: the encode sizing / packing and decode loops of the
// real kernels (included below) run R times on a tile staged once in each
// wave's LDS region -- no look-back, no global traffic in the timed loop.
// Prints cycles per tile per wave for each phase.  Build:
//   hipcc -O3 --offload-arch=gfx950 -I../../ls-qpack_amd/csrc codec_bench.hip
#include "../../ls-qpack_amd/csrc/qhuff_encode.hip"
#include "../../ls-qpack_amd/csrc/qhuff_decode.hip"
#include "../../ls-qpack_amd/csrc/qhuff_tables.cpp"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

using namespace qhuff;

#ifndef MB_WAVES
#define MB_WAVES 12
#endif

struct MbOut { unsigned long long cyc[4]; unsigned long long sum; };

template <int W>
__global__ __launch_bounds__(64 * W) void
mb_encode(EncArgs a, int reps, MbOut *res)
{
    __shared__ EncSmem smem;
    QH_LDS EncSmem *sm = (QH_LDS EncSmem *) &smem;
    const int tid = threadIdx.x;
    enc_tables_load(sm, a.enc, tid);
    __syncthreads();
    QH_LDS EncWave *wv = &sm->w[tid >> 6];
    const uint32_t gid = blockIdx.x * W + (tid >> 6), lane = lane_id();
    const uint32_t t = gid % a.c.n_tiles;
    TileOffs to;
    to.load((const QH_GLB uint32_t *) a.in_off, (uint64_t) t * kWT, kWT);
    const Span sp = tile_span(a.in, to.first(), to.last(), kStageCap);
    Chunks<kChunks> ch;
    ch.load(sp);
    EncPolicy pol;
    pol.in = a.in;
    pol.mode = a.mode;
    pol.sm = sm;
    pol.wv = wv;
    unsigned long long c0 = 0, c1 = 0, sum = 0;
    for (int r = 0; r < reps; ++r)
    {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        pol.stage_in(ch, sp, to);
        wave_sync();
        pol.prepare(sp);                     // the encoder's dense pass
        uint32_t sz, st;
        pol.codec(to, kWT, sp, &sz, &st);
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t total = read_lane(incl, 63);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        wave_sync();
        pol.emit(incl - sz, sz, total);
        wave_sync();
        sum += wv->out[lane] + total;
        const uint64_t t2 = __builtin_amdgcn_s_memtime();
        c0 += t1 - t0;
        c1 += t2 - t1;
    }
    if (lane == 0)
    {
        res[gid].cyc[0] = c0 / reps;
        res[gid].cyc[1] = c1 / reps;
        res[gid].sum = sum;
    }
}

template <int W>
__global__ __launch_bounds__(64 * W) void
mb_decode(DecArgs a, int reps, MbOut *res)
{
    __shared__ DecSmem smem;
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    const int tid = threadIdx.x;
    {
        const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) a.win;
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
        for (int i = tid; i < kWinSize / 4; i += 64 * W)
            sw[i] = gw[i];
        if (tid < 257)
            sm->sorted[tid] = a.sorted[tid];
    }
    __syncthreads();
    QH_LDS DecWave *wv = &sm->w[tid >> 6];
    const uint32_t gid = blockIdx.x * W + (tid >> 6), lane = lane_id();
    const uint32_t t = gid % a.c.n_tiles;
    TileOffs to;
    to.load((const QH_GLB uint32_t *) a.in_off, (uint64_t) t * kWT, kWT);
    const Span sp = tile_span(a.in, to.first(), to.last(), kStageCap);
    Chunks<kChunks> ch;
    ch.load(sp);
    DecPolicy pol{a.in, sm, wv, 0};
    unsigned long long c0 = 0, c1 = 0, sum = 0;
    for (int r = 0; r < reps; ++r)
    {
        ch.store<true>((QH_LDS u32x4 *) wv->in, sp.n16);   // emit overwrites it
        wave_sync();
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        uint32_t sz, st;
        pol.codec(to, kWT, sp, &sz, &st);
        const uint32_t incl = wave_incl_scan(sz);
        const uint32_t total = read_lane(incl, 63);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        wave_sync();
        pol.emit(incl - sz, sz, total);
        wave_sync();
        sum += wv->in[lane] + total + st;
        const uint64_t t2 = __builtin_amdgcn_s_memtime();
        c0 += t1 - t0;
        c1 += t2 - t1;
    }
    if (lane == 0)
    {
        res[gid].cyc[0] = c0 / reps;
        res[gid].cyc[1] = c1 / reps;
        res[gid].sum = sum;
    }
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

// host Huffman encode (payload) for the decode input
static void henc(const HostTables &t, const std::vector<uint8_t> &d,
                 const std::vector<uint32_t> &off, std::vector<uint8_t> &h,
                 std::vector<uint32_t> &ho)
{
    const uint32_t n = off.size() - 1;
    ho.resize(n + 1);
    h.clear();
    for (uint32_t i = 0; i < n; ++i)
    {
        ho[i] = h.size();
        uint64_t acc = 0; int nb = 0;
        for (uint32_t k = off[i]; k < off[i + 1]; ++k)
        {
            acc = (acc << t.bits[d[k]]) | t.code[d[k]];
            nb += t.bits[d[k]];
            while (nb >= 8) { h.push_back((uint8_t) (acc >> (nb - 8))); nb -= 8; }
        }
        if (nb) h.push_back((uint8_t) ((acc << (8 - nb)) | ((1u << (8 - nb)) - 1)));
    }
    ho[n] = h.size();
}

template <class F>
static void report(const char *tag, F launch, int nw)
{
    MbOut *d;
    hipMalloc(&d, sizeof(MbOut) * nw);
    for (int rep = 0; rep < 2; ++rep)
        launch(d);
    hipDeviceSynchronize();
    std::vector<MbOut> h(nw);
    hipMemcpy(h.data(), d, sizeof(MbOut) * nw, hipMemcpyDeviceToHost);
    double a = 0, b = 0;
    for (auto &x : h) { a += x.cyc[0]; b += x.cyc[1]; }
    printf("%-28s codec+scan %7.0f   emit %7.0f  cycles/tile/wave (%d waves)\n",
           tag, a / nw, b / nw, nw);
    hipFree(d);
}

int main(int argc, char **argv)
{
    const uint32_t n = 1 << 20;
    std::vector<uint8_t> data, hd;
    std::vector<uint32_t> off, ho;
    synth(n, data, off);
    HostTables ht;
    build_tables(&ht);
    henc(ht, data, off, hd, ho);
    uint8_t *d_in, *d_h;
    uint32_t *d_off, *d_ho, *d_win;
    uint2 *d_enc;
    uint16_t *d_sorted;
    hipMalloc(&d_in, data.size() + 64);
    hipMalloc(&d_h, hd.size() + 64);
    hipMalloc(&d_off, 4 * (n + 1));
    hipMalloc(&d_ho, 4 * (n + 1));
    hipMalloc(&d_win, sizeof(ht.win));
    hipMalloc(&d_enc, 8 * 257);
    hipMalloc(&d_sorted, 2 * 257);
    hipMemcpy(d_in, data.data(), data.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_h, hd.data(), hd.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_off, off.data(), 4 * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(d_ho, ho.data(), 4 * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(d_win, ht.win, sizeof(ht.win), hipMemcpyHostToDevice);
    std::vector<uint2> enc(257);
    for (int i = 0; i < 257; ++i) enc[i] = make_uint2(ht.code[i], ht.bits[i]);
    hipMemcpy(d_enc, enc.data(), 8 * 257, hipMemcpyHostToDevice);
    hipMemcpy(d_sorted, ht.sorted, 2 * 257, hipMemcpyHostToDevice);
    const int reps = argc > 1 ? atoi(argv[1]) : 64;
    const int blocks = 256;
    {
        EncArgs a = {};
        a.in = d_in; a.in_off = d_off; a.enc = d_enc; a.n = n; a.mode = 0;
        a.c.n_tiles = n / 64;
        report("encode (12 waves/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_encode<12>, dim3(blocks), dim3(768), 0, 0, a, reps, r); },
            blocks * 12);
        report("encode (4 waves/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_encode<4>, dim3(blocks), dim3(256), 0, 0, a, reps, r); },
            blocks * 4);
        report("encode (1 wave/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_encode<1>, dim3(blocks), dim3(64), 0, 0, a, reps, r); },
            blocks * 1);
    }
    {
        DecArgs a = {};
        a.in = d_h; a.in_off = d_ho; a.win = d_win; a.sorted = d_sorted; a.n = n;
        a.c.n_tiles = n / 64;
        report("decode (12 waves/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_decode<12>, dim3(blocks), dim3(768), 0, 0, a, reps, r); },
            blocks * 12);
        report("decode (4 waves/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_decode<4>, dim3(blocks), dim3(256), 0, 0, a, reps, r); },
            blocks * 4);
        report("decode (1 wave/CU)", [&](MbOut *r) {
            hipLaunchKernelGGL(mb_decode<1>, dim3(blocks), dim3(64), 0, 0, a, reps, r); },
            blocks * 1);
    }
    return 0;
}
