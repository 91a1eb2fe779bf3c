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
// One string per lane, one 64-string tile per wave (qhuff_device.h).  The
// tile's Huffman input is staged in the wave's LDS region as big-endian
// dwords.  Each lane holds its bit stream as two dwords A:B and a bit
// position (decode_string_lds): a step looks the next 13 bits up in a window
// table (up to two symbols of <= 13 bits), writes the entry's two symbol
// bytes to the string's arena slot and advances by the bits consumed.
// Codes of 14..30 bits stall their lane and are decoded together outside the
// step loop by a canonical length search.  Main steps run while the lane has
// >= 13 real bits; the last < 13 bits (at most two symbols) take a padded
// one-lookup epilogue that applies the D3 tail rule (fewer than 8 padding
// bits, all ones).
//
// After the wave scan of the output sizes the arena slots are compacted
// into the (now dead) input stage and copied out with 16-byte stores once
// the look-back has resolved the tile's output base.
#include "qhuff_decode_impl.h"

#include <hip/hip_ext.h>

// tickets claimed per wave in the prologue, at most (see qhuff_encode.hip)
#ifndef QH_DEC_PER
#define QH_DEC_PER 2
#endif

namespace qhuff {

// Keep: the per-string entry points' kernel (DecPolicyT); a template
// parameter, so the batch kernel's code and registers are untouched
template <bool Keep, bool Full>
__global__ __launch_bounds__(64 * kWaves) void
qhuff_decode_kernel(DecArgs a)
{
    __shared__ DecSmem smem;
    QH_LDS DecSmem *sm = (QH_LDS DecSmem *) &smem;
    const int tid = threadIdx.x;
    prof_realtime(a.c, kProfIters - 1, 10);      // (profiling) wave entry
    Tickets tk;
    tk.init();
    // The workgroup's ticket claims go out first, then every load of the
    // tables; the claims are waited for (not the tables) and shared at the
    // first barrier, each wave then issues its first offsets loads, and only
    // then are the tables stored and the second barrier passed (in
    // tile_pipeline's mid()): the offsets loads overlap the table loads.
    const uint32_t cb = claim_block_issue(a.c, tk, QH_DEC_PER);
    constexpr int kPer = (kWinSize / 4 + 64 * kWaves - 1) / (64 * kWaves);
    const QH_GLB u32x4 *gw = (const QH_GLB u32x4 *) glb(a.win);
    u32x4 v[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r)
    {
        const int i = tid + r * 64 * kWaves;
        v[r] = gw[i < kWinSize / 4 ? i : 0];
    }
    const QH_GLB uint16_t *gs = glb(a.sorted);
    const uint16_t so = gs[tid < 257 ? tid : 0];
    static_assert(kLong2Size <= 64 * kWaves, "one long2 entry per thread");
    const uint16_t l2 = glb(a.long2)[tid < kLong2Size ? tid : 0];
    claim_block_store(a.c, cb, &sm->tk, QH_DEC_PER);
    clear_next_launch(a.c);
    // the tickets: LDS stores visible, no wait for the table loads (a
    // __syncthreads() would drain them)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    prof_realtime(a.c, kProfIters - 1, 11);      // (profiling) after it
    DecPolicyT<DecSmem, Keep, Full> pol{a.in, sm,
                                  &sm->w[__builtin_amdgcn_readfirstlane(tid >> 6)], 0};
#ifdef QHUFF_PROFILE
    pol.pc = &a.c;
#endif
    uint32_t t0, k1, k2;
    wave_tickets(a.c, tk, &sm->tk, &t0, &k1, &k2);
    auto tables = [&]() {
        QH_LDS u32x4 *sw = (QH_LDS u32x4 *) sm->win;
#pragma unroll
        for (int r = 0; r < kPer; ++r)
        {
            const int i = tid + r * 64 * kWaves;
            if (i < kWinSize / 4)
                sw[i] = v[r];
        }
        if (tid < 257)
            sm->sorted[tid] = so;
        if (tid < kLong2Size)
            sm->long2[tid] = l2;
        if (tid == 0)
            sm->win[kHoldIdx] = kHoldEntry;
        __syncthreads();             // the tables
    };
    tile_pipeline(pol, a.c, tk, t0, k1, k2, a.in, a.in_off,
                  a.n, a.out, a.out_off, a.status, tables);
}

hipError_t
launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st, hipEvent_t ev0,
              hipEvent_t ev1, bool keep, bool full)
{
    if (keep)
        hipLaunchKernelGGL((qhuff_decode_kernel<true, false>), dim3(grid),
                           dim3(64 * kWaves), 0, st, a);
    else if (full && ev0)
        hipExtLaunchKernelGGL((qhuff_decode_kernel<false, true>), dim3(grid),
                              dim3(64 * kWaves), 0, st, ev0, ev1, 0, a);
    else if (full)
        hipLaunchKernelGGL((qhuff_decode_kernel<false, true>), dim3(grid),
                           dim3(64 * kWaves), 0, st, a);
    else if (ev0)
        hipExtLaunchKernelGGL((qhuff_decode_kernel<false, false>), dim3(grid),
                              dim3(64 * kWaves), 0, st, ev0, ev1, 0, a);
    else
        hipLaunchKernelGGL((qhuff_decode_kernel<false, false>), dim3(grid),
                           dim3(64 * kWaves), 0, st, a);
    return hipGetLastError();
}

hipError_t
decode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_decode_kernel<false, true>),
        64 * kWaves, 0);
}

int
decode_waves_per_block()
{
    return kWaves;
}

uint32_t
decode_tile_strings()
{
    return kDecTS;
}

size_t
decode_lds_bytes()
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(qhuff_decode_kernel<false, true>))
            != hipSuccess)
        return 0;
    return fa.sharedSizeBytes;
}

}  // namespace qhuff
