// Decode step-loop lab: decode_string_lds (the real kernel's codec, included
// below) run R times on a tile staged once in each wave's LDS region, with
// different output sinks, at 1 / 4 / 8 / 12 waves per CU.  Separates the
// cost of the step's byte stores from its lookup / refill chain.  Prints
// cycles per tile per wave and per wave-step.  Build:
//   hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None step_lab.hip
#include "../../ls-qpack_amd/csrc/qhuff_decode.hip"
#include "../../ls-qpack_amd/csrc/qhuff_tables.cpp"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

using namespace qhuff;

struct NullEmit                       // counts only: no LDS store
{
    uint32_t n;
    uint32_t k;
    __device__ __forceinline__ void finish() {}
    __device__ __forceinline__ void operator()(uint32_t, uint32_t nb)
    {
        n += nb;
    }
};

// one aligned 16-bit record per step (sym0, sym1) at a lane-major address
// advanced by 2 per step: one ds_write_b16 instead of two ds_write_b8
struct RecEmit
{
    QH_LDS uint16_t *p;
    uint32_t n;
    __device__ __forceinline__ void finish() {}
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        *p = (uint16_t) __builtin_amdgcn_perm(val, val, 0x0c0c0200u);
        p += 1;
        n += nb;
    }
};

// one byte store per step (sym0 only): half the stores of ArenaEmit
struct OneByteEmit
{
    QH_LDS uint8_t *slot, *p;
    uint32_t n;
    __device__ __forceinline__ void finish() { n = (uint32_t) (p - slot); }
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        p[0] = (uint8_t) val;
        p += nb;
    }
};

// both symbol bytes with ONE ds_write_b16 at the byte address p (unaligned
// when p is odd; crosses a dword when p % 4 == 3)
struct U16Emit
{
    QH_LDS uint8_t *slot, *p;
    uint32_t n;
    __device__ __forceinline__ void finish() { n = (uint32_t) (p - slot); }
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        *(QH_LDS uint16_t *) p =
            (uint16_t) __builtin_amdgcn_perm(val, val, 0x0c0c0200u);
        p += nb;
    }
};

// the window entry itself, one ds_write_addtid_b32 per step into a
// step-major arena (address M0 + 4 * lane, no address VGPR; M0 moves on
// 256 B per step, wrapping in 4 KB: timing only, the bytes are not kept)
struct AddtidEmit
{
    uint32_t base;                   // wave's arena byte address (uniform)
    uint32_t step;                   // uniform step counter
    uint32_t n;
    __device__ __forceinline__ void finish() {}
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(base + ((step & 15u) << 8));
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tds_write_addtid_b32 %0"
                     : : "v"(val), "s"(m0) : "m0", "memory");
        ++step;
        n += nb;
    }
};

//  each lane's output bytes packed in a register and
// written one dword at a time: every step ORs its nb bytes into the dword
// being filled and stores that dword (partial or full, ONE ds_write_b32 per
// step instead of two ds_write_b8), moving on a dword when it is full.  The
// lane's slot must start on a dword (sl % 4 == 0).
struct PackEmit
{
    QH_LDS uint32_t *slot, *p;
    uint32_t acc;                    // bytes of *p so far (sh / 8 of them)
    uint32_t sh;                     // 8 * bytes in acc
    uint32_t n;
    __device__ __forceinline__ void finish() {}
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        // sym0 [7:0], sym1 [23:16] -> bytes 0, 1; only nb of them
        uint32_t two = __builtin_amdgcn_perm(val, val, 0x0c0c0200u);
        two = __builtin_amdgcn_ubfe(two, 0, 8 * nb);
        const uint32_t v = acc | (two << sh);
        *p = v;
        const uint32_t s2 = sh + 8 * nb;
        const bool full = s2 >= 32;
        const uint32_t carry = sh ? two >> ((32 - sh) & 31) : 0u;
        acc = full ? carry : v;
        p += full ? 1 : 0;
        sh = s2 & 31;
        n += nb;
    }
};
// the same, the store only when the dword is full (exec-masked), the
// partial dword once at the end
struct PackEmitM
{
    QH_LDS uint32_t *slot, *p;
    uint32_t acc, sh, n;
    __device__ __forceinline__ void finish()
    {
        if (sh)
            *p = acc;
    }
    __device__ __forceinline__ void operator()(uint32_t val, uint32_t nb)
    {
        uint32_t two = __builtin_amdgcn_perm(val, val, 0x0c0c0200u);
        two = __builtin_amdgcn_ubfe(two, 0, 8 * nb);
        const uint32_t v = acc | (two << sh);
        const uint32_t s2 = sh + 8 * nb;
        const bool full = s2 >= 32;
        if (full)
            *p = v;
        const uint32_t carry = sh ? two >> ((32 - sh) & 31) : 0u;
        acc = full ? carry : v;
        p += full ? 1 : 0;
        sh = s2 & 31;
        n += nb;
    }
};

struct MbOut { unsigned long long cyc, steps, sum; };

template <int W, int MODE>
__global__ __launch_bounds__(64 * W) void
lab(DecArgs a, int reps, MbOut *res)
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
        if (tid == 0)
            sm->win[kHoldIdx] = kHoldEntry;
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
    ch.store<true>((QH_LDS u32x4 *) wv->in, sp.n16);
    wave_sync();
    const uint32_t A0 = to.first();
    const uint32_t slot0 = 2 * lane + (uint32_t) ((8ull * (to.o0 - A0)) / 5);
    const uint32_t rs = (uint32_t) ((uintptr_t) (a.in + to.o0) - sp.pa);
    const uint32_t re = (uint32_t) ((uintptr_t) (a.in + to.o1) - sp.pa);
    unsigned long long c0 = 0, sum = 0;
    for (int r = 0; r < reps; ++r)
    {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        int n;
        if (MODE == 0)
        {
            ArenaEmit em{wv->arena + slot0, wv->arena + slot0, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 1)
        {
            NullEmit em{0, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 2)
        {
            // lane-major records: lane l's at arena + 76 * l (76 B = 19
            // dwords, odd: the 32 lanes of a group on distinct banks)
            RecEmit em{(QH_LDS uint16_t *) (wv->arena + 76 * lane), 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 3)
        {
            OneByteEmit em{wv->arena + slot0, wv->arena + slot0, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 7 || MODE == 8)
        {
            const uint32_t sl = MODE == 7 ? slot0 : 84 * lane;
            U16Emit em{wv->arena + sl, wv->arena + sl, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 9 || MODE == 10)
        {
            // the kernel's sink (fixed stride 108), one refill read per step
            // (9) or per two steps (10, QH_REFILL2)
            ArenaEmit em{wv->arena + 108 * lane, wv->arena + 108 * lane, 0};
            n = MODE == 9
                ? decode_string_lds<ArenaEmit, false>(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em)
                : decode_string_lds<ArenaEmit, true>(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else if (MODE == 12 || MODE == 13 || MODE == 14 || MODE == 15)
        {
            // packed dwords: fixed stride 108 (12, 13) or the kernel's
            // variable slots rounded up to a dword (14, 15; 4 bytes of
            // slack per lane instead of 2)
            const uint32_t sl = MODE <= 13 ? 108 * lane
                              : (4 * lane + (uint32_t) ((8ull * (to.o0 - A0)) / 5) + 3) & ~3u;
            QH_LDS uint32_t *q = (QH_LDS uint32_t *) (wv->arena + sl);
            if (MODE == 12 || MODE == 14)
            {
                PackEmit em{q, q, 0, 0, 0};
                n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
            }
            else
            {
                PackEmitM em{q, q, 0, 0, 0};
                n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
            }
        }
        else if (MODE == 16)
        {
            // the kernel's sink in the kernel's variable slots
            ArenaEmit em{wv->arena + slot0, wv->arena + slot0, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        else
        {
            // the kernel's two byte stores into a fixed-stride lane-major
            // arena: lane l's slot at STRIDE * l (an odd number of dwords:
            // lanes at equal progress on distinct banks)
            constexpr uint32_t STRIDE = MODE == 4 ? 84 : MODE == 5 ? 76 : 68;
            ArenaEmit em{wv->arena + STRIDE * lane, wv->arena + STRIDE * lane, 0};
            n = decode_string_lds(wv->in, 8 * rs, 8 * re, sm->win, sm->sorted, sm->long2, em);
        }
        sum += read_lane((uint32_t) n, 63);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        c0 += t1 - t0;
        wave_sync();
    }
    // steps of this tile: the longest string's bits / ~11.7 is not exact;
    // report bits of the longest string instead
    const uint32_t bits = wave_max(8 * (re - rs));
    if (lane == 0)
    {
        res[gid].cyc = c0 / reps;
        res[gid].steps = bits;
        res[gid].sum = sum;
    }
}

// MODE 11 layout: the step-major arenas first (M0[15:0] addresses the
// first 64 KB only), then the tables and the input stages
template <int W>
struct AddtidSmem
{
    uint32_t arena[W][1024];                 // 16 steps x 64 lanes x 4 B
    uint32_t win[kWinSize + 4];
    uint16_t sorted[257];
    uint16_t long2[kLong2Size];   // (not loaded: the lab strings have no long codes)
    alignas(16) uint32_t in[W][kDecStageCap / 4];
};

template <int W>
__global__ __launch_bounds__(64 * W) void
lab_addtid(DecArgs a, int reps, MbOut *res)
{
    __shared__ AddtidSmem<W> smem;
    QH_LDS AddtidSmem<W> *sm = (QH_LDS AddtidSmem<W> *) &smem;
    const int tid = threadIdx.x;
    for (int i = tid; i < kWinSize; i += 64 * W)
        sm->win[i] = a.win[i];
    if (tid < 257)
        sm->sorted[tid] = a.sorted[tid];
    if (tid == 0)
        sm->win[kHoldIdx] = kHoldEntry;
    __syncthreads();
    const uint32_t w = tid >> 6;
    const uint32_t gid = blockIdx.x * W + w, lane = lane_id();
    const uint32_t t = gid % a.c.n_tiles;
    TileOffs to;
    to.load((const QH_GLB uint32_t *) a.in_off, (uint64_t) t * kWT, kWT);
    const Span sp = tile_span(a.in, to.first(), to.last(), kStageCap);
    Chunks<kChunks> ch;
    ch.load(sp);
    ch.store<true>((QH_LDS u32x4 *) sm->in[w], sp.n16);
    wave_sync();
    const uint32_t rs = (uint32_t) ((uintptr_t) (a.in + to.o0) - sp.pa);
    const uint32_t re = (uint32_t) ((uintptr_t) (a.in + to.o1) - sp.pa);
    const uint32_t base = (uint32_t) (uintptr_t) &sm->arena[w][0];
    unsigned long long c0 = 0, sum = 0;
    for (int r = 0; r < reps; ++r)
    {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        AddtidEmit em{(uint32_t) __builtin_amdgcn_readfirstlane((int) base), 0, 0};
        int n = decode_string_lds(sm->in[w], 8 * rs, 8 * re, sm->win,
                                  sm->sorted, sm->long2, em);
        sum += read_lane((uint32_t) n, 63);
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        c0 += t1 - t0;
        wave_sync();
    }
    const uint32_t bits = wave_max(8 * (re - rs));
    if (lane == 0)
    {
        res[gid].cyc = c0 / reps;
        res[gid].steps = bits;
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

template <int W>
static void run_addtid(const char *tag, const DecArgs &a, int reps)
{
    const int blocks = 256, nw = blocks * W;
    MbOut *d;
    hipMalloc(&d, sizeof(MbOut) * nw);
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((lab_addtid<W>), dim3(blocks), dim3(64 * W), 0, 0,
                           a, reps, d);
    hipDeviceSynchronize();
    std::vector<MbOut> h(nw);
    hipMemcpy(h.data(), d, sizeof(MbOut) * nw, hipMemcpyDeviceToHost);
    double cyc = 0, bits = 0;
    for (auto &x : h) { cyc += x.cyc; bits += x.steps; }
    cyc /= nw;
    bits /= nw;
    printf("%-14s %2d waves/CU: %7.0f cycles/tile/wave  %5.0f cycles per "
           "step (max string %4.0f bits)\n", tag, W, cyc, cyc / (bits / 11.6),
           bits);
    hipFree(d);
}

template <int W, int MODE>
static void run(const char *tag, const DecArgs &a, int reps)
{
    const int blocks = 256, nw = blocks * W;
    MbOut *d;
    hipMalloc(&d, sizeof(MbOut) * nw);
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL((lab<W, MODE>), dim3(blocks), dim3(64 * W), 0, 0, a,
                           reps, d);
    hipDeviceSynchronize();
    std::vector<MbOut> h(nw);
    hipMemcpy(h.data(), d, sizeof(MbOut) * nw, hipMemcpyDeviceToHost);
    double cyc = 0, bits = 0;
    for (auto &x : h) { cyc += x.cyc; bits += x.steps; }
    cyc /= nw;
    bits /= nw;
    // steps ~ longest string bits / 11.6 (13-bit window, token alphabet)
    printf("%-14s %2d waves/CU: %7.0f cycles/tile/wave  %5.0f cycles per "
           "step (max string %4.0f bits)\n", tag, W, cyc, cyc / (bits / 11.6),
           bits);
    hipFree(d);
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    const uint32_t n = 1 << 20;
    std::vector<uint8_t> data, hd;
    std::vector<uint32_t> off, ho;
    synth(n, data, off);
    HostTables ht;
    build_tables(&ht);
    henc(ht, data, off, hd, ho);
    uint8_t *d_h;
    uint32_t *d_ho, *d_win;
    uint16_t *d_sorted;
    hipMalloc(&d_h, hd.size() + 64);
    hipMalloc(&d_ho, 4 * (n + 1));
    hipMalloc(&d_win, sizeof(ht.win));
    hipMalloc(&d_sorted, 2 * 257);
    hipMemcpy(d_h, hd.data(), hd.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_ho, ho.data(), 4 * (n + 1), hipMemcpyHostToDevice);
    hipMemcpy(d_win, ht.win, sizeof(ht.win), hipMemcpyHostToDevice);
    hipMemcpy(d_sorted, ht.sorted, 2 * 257, hipMemcpyHostToDevice);
    const int reps = argc > 1 ? atoi(argv[1]) : 64;
    DecArgs a = {};
    a.in = d_h; a.in_off = d_ho; a.win = d_win; a.sorted = d_sorted; a.n = n;
    a.c.n_tiles = n / 64;
    if (argc > 2 && argv[2][0] == 'p')
    {
        // the packed-dword sink against the kernel's,
        // interleaved
        for (int k = 0; k < 3; ++k)
        {
            run<12, 16>("arena b8x2 var", a, reps);
            run<12, 14>("pack b32 var", a, reps);
            run<12, 15>("packM b32 var", a, reps);
            run<12, 10>("arena b8x2 108", a, reps);
            run<12, 12>("pack b32 108", a, reps);
            run<12, 13>("packM b32 108", a, reps);
            run<12, 1>("no store", a, reps);
        }
        return 0;
    }
    if (argc > 2)
    {
        // the refill A/B only, interleaved
        for (int k = 0; k < 3; ++k)
        {
            run<1, 9>("fixed108 r1", a, reps);
            run<1, 10>("fixed108 r2", a, reps);
            run<8, 9>("fixed108 r1", a, reps);
            run<8, 10>("fixed108 r2", a, reps);
            run<12, 9>("fixed108 r1", a, reps);
            run<12, 10>("fixed108 r2", a, reps);
        }
        return 0;
    }
    run<1, 0>("arena b8x2", a, reps);
    run<4, 0>("arena b8x2", a, reps);
    run<8, 0>("arena b8x2", a, reps);
    run<12, 0>("arena b8x2", a, reps);
    run<1, 1>("no store", a, reps);
    run<4, 1>("no store", a, reps);
    run<8, 1>("no store", a, reps);
    run<12, 1>("no store", a, reps);
    run<1, 2>("record b16", a, reps);
    run<4, 2>("record b16", a, reps);
    run<8, 2>("record b16", a, reps);
    run<12, 2>("record b16", a, reps);
    run<1, 3>("one b8", a, reps);
    run<12, 3>("one b8", a, reps);
    run<1, 4>("fixed 84", a, reps);
    run<8, 4>("fixed 84", a, reps);
    run<12, 4>("fixed 84", a, reps);
    run<12, 5>("fixed 76", a, reps);
    run<12, 6>("fixed 68", a, reps);
    run_addtid<1>("addtid u32", a, reps);
    run_addtid<8>("addtid u32", a, reps);
    run_addtid<12>("addtid u32", a, reps);
    run<1, 7>("u16 unaligned", a, reps);
    run<12, 7>("u16 unaligned", a, reps);
    run<12, 8>("u16 fixed 84", a, reps);
    return 0;
}
