// qhuff_encode.hip -- batch Huffman encode kernel (gfx950).
//
// Reference path:
//   E1 qenc_enc_str_size   lsqpack.c:5198-5210  -> sizing
//   E2 qenc_huffman_enc    lsqpack.c:5085-5195  -> packing
//   E3 lsqpack_enc_enc_str lsqpack.c:839-876    -> LITERAL modes (H bit,
//                          prefixed length, strict-< Huffman-vs-raw choice)
//
// One 64-string tile per wave (qhuff_device.h, qhuff_pipeline.h).  The
// tile's packed input arrives as 16-byte chunks in registers (lane l holds
// chunks l, l + 64, l + 128 of the tile's 16-byte aligned span).  Per tile:
//   1. dense pass, byte-parallel (no per-string work, no divergence): each
//      lane looks up the codes of its 16 bytes per row (one LDS read per
//      byte), the row's lane sums are scanned across the wave, and the codes
//      are OR-ed four at a time into a dense bit stream -- the codes of every
//      byte of the span back to back, with no padding or framing.  Each
//      byte's code length (u8) and each chunk's dense offset stay in LDS;
//   2. sizing, string per lane: a string's Huffman bits (E1) are the
//      difference of the dense offsets of its two ends -- a chunk offset
//      plus a SAD over at most 16 byte lengths each; the E3 choice; wave
//      scan -> tile-local output offsets;
//   3. emit, string per lane: framing bits, the string's range of the dense
//      stream funnel-copied word by word to its byte-aligned output position,
//      EOS-prefix padding (lsqpack.c:5171-5189); raw strings copied from the
//      staged input;
//   4. look-back for the tile's global output base, 16-byte stores
//      (qhuff_pipeline.h).
// A tile whose dense stream overflows its buffer is sized and packed string
// per lane from the staged input instead (codes of any length go into the
// dense stream); tiles that do not fit the stages are big tiles
// (qhuff_pipeline.h).
#include "qhuff_encode_impl.h"

#include <hip/hip_ext.h>

// tickets claimed per wave in the prologue, at most (tile_pipeline).  2: the
// third and fourth tickets are claimed by each wave at its first top, after
// every workgroup's first claims (tile_pipeline `late`).  3 (round 3,
// profiles/r03_ep3) put every workgroup's third tiles ahead of later
// workgroups' first ones, and the first flush waited for the slowest of
// them (profiles/r04_r; r04_s: first flush 10.4k -> 3.1k cycles).
#ifndef QH_ENC_PER
#define QH_ENC_PER 2
#endif

namespace qhuff {

template <bool Full>
__global__ __launch_bounds__(64 * kWaves) void
qhuff_encode_kernel(EncArgs a)
{
    __shared__ EncSmem smem;
    QH_LDS EncSmem *sm = (QH_LDS EncSmem *) &smem;
    const int tid = threadIdx.x;
    Tickets tk;
    tk.init();
    // the ticket atomics go out first (they queue behind every other
    // workgroup's on the counters), then the table loads
    const uint32_t cb = claim_block_issue(a.c, tk, QH_ENC_PER);
    enc_tables_load(sm, a.enc, tid);
    claim_block_store(a.c, cb, &sm->tk, QH_ENC_PER);
    clear_next_launch(a.c);
    __syncthreads();                 // the only workgroup barrier
    EncPolicyT<EncSmem, Full> pol;
    pol.in = a.in;
    pol.mode = a.mode;
    pol.sm = sm;
    pol.wv = &sm->w[__builtin_amdgcn_readfirstlane(tid >> 6)];
    pol.dense = false;
    uint32_t t0, k1, k2;
    wave_tickets(a.c, tk, &sm->tk, &t0, &k1, &k2);
    tile_pipeline(pol, a.c, tk, t0, k1, k2, a.in, a.in_off,
                  a.n, a.out, a.out_off, nullptr);
}

hipError_t
launch_encode(const EncArgs &a, uint32_t grid, hipStream_t st, hipEvent_t ev0,
              hipEvent_t ev1, bool full)
{
    if (full && ev0)
        hipExtLaunchKernelGGL(qhuff_encode_kernel<true>, dim3(grid),
                              dim3(64 * kWaves), 0, st, ev0, ev1, 0, a);
    else if (full)
        hipLaunchKernelGGL(qhuff_encode_kernel<true>, dim3(grid),
                           dim3(64 * kWaves), 0, st, a);
    else if (ev0)
        hipExtLaunchKernelGGL(qhuff_encode_kernel<false>, dim3(grid),
                              dim3(64 * kWaves), 0, st, ev0, ev1, 0, a);
    else
        hipLaunchKernelGGL(qhuff_encode_kernel<false>, dim3(grid),
                           dim3(64 * kWaves), 0, st, a);
    return hipGetLastError();
}

hipError_t
encode_occupancy(int *blocks_per_cu)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        blocks_per_cu, reinterpret_cast<const void *>(qhuff_encode_kernel<true>),
        64 * kWaves, 0);
}

int
encode_waves_per_block()
{
    return kWaves;
}

size_t
encode_lds_bytes()
{
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(qhuff_encode_kernel<true>))
            != hipSuccess)
        return 0;
    return fa.sharedSizeBytes;
}

}  // namespace qhuff
