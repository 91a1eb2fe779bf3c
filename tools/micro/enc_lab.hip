// Encode phase lab: the real kernel's dense pass, sizing and emit
// (qhuff_encode.hip) run R times on a tile staged once in each wave's LDS
// region, at 1 and 12 waves per CU.  Prints cycles per tile per wave for
// each phase.  Build:
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None enc_lab.hip
#include "../../ls-qpack_amd/csrc/qhuff_encode.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

using namespace qhuff;

struct MbOut { unsigned long long c_dense, c_size, c_emit, sum; };

template <int W>
__global__ __launch_bounds__(64 * W) void
enc_lab(EncArgs a, int reps, MbOut *res)
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
    EncPolicyT<EncSmem, false> pol;
    pol.in = a.in;
    pol.mode = a.mode;
    pol.sm = sm;
    pol.wv = wv;
    pol.dense = false;
    pol.stage_in(ch, sp, to);
    wave_sync();
    unsigned long long cd = 0, cs = 0, ce = 0, sum = 0;
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
        pol.emit(incl - sz, sz, total);
        wave_sync();
        sum += wv->out[lane] + total + (pol.dense ? 1 : 0);
        const uint64_t t3 = __builtin_amdgcn_s_memtime();
        cd += t1 - t0;
        cs += t2 - t1;
        ce += t3 - t2;
    }
    if (lane == 0)
    {
        res[gid].c_dense = cd / reps;
        res[gid].c_size = cs / reps;
        res[gid].c_emit = ce / reps;
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
    double x = 0, y = 0, z = 0;
    for (auto &o : h) { x += o.c_dense; y += o.c_size; z += o.c_emit; }
    printf("%2d waves/CU: dense %6.0f  sizing+scan %6.0f  emit %6.0f  "
           "cycles/tile/wave\n", W, x / nw, y / nw, z / nw);
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
