// qhuff_kernels.h -- argument blocks and launch entry points shared by the
// kernel translation units and the host C-ABI (qhuff_host.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qhuff.h"
#include "qhuff_device.h"
#include "qhuff_tables.h"

namespace qhuff {

struct LongParams
{
    LongLen l[kMaxLong];
    uint32_t n;
};

struct EncArgs
{
    const uint8_t *in;
    const uint32_t *in_off;
    uint8_t *out;
    uint32_t *out_off;
    const uint2 *enc;            // 257 x {code, bits}
    uint64_t n;
    uint32_t mode;               // 0 payload, 3/5/7 literal prefix bits
    Coord c;
};

struct DecArgs
{
    const uint8_t *in;
    const uint32_t *in_off;
    uint8_t *out;
    uint32_t *out_off;
    uint8_t *status;
    const uint32_t *win;         // kWinSize window entries
    const uint16_t *sorted;      // 257 symbols in canonical order
    const uint16_t *long2;       // kLong2Size long codes by leading ones
    uint64_t n;
    Coord c;
    LongParams lp;
};

struct HashArgs
{
    const uint8_t *in;
    const uint32_t *off;         // pairs: 2n + 1 offsets, else n + 1
    uint32_t *h1;                // name hash (pairs) / string hash
    uint32_t *h2;                // name+value hash (pairs only)
    uint64_t n;
    uint32_t seed;
    uint32_t pairs;
};

// ---- low-latency service (qhuff_service.hip, qhuff_svc_* in qhuff_host.cpp)
//
// One request slot per service wave, in pinned host memory mapped into the
// device (fine-grained): the host writes a request and then its sequence
// number; the wave polls that word, codes the request and writes the result
// back into the slot, then the done word.  Slot layout (bytes):
//   header      kSvcHdrBytes   (SvcHdr)
//   in_off      (n + 1) u32, rebased to 0
//   in          the request's bytes
//   out_off     (n + 1) u32
//   status      n u8 (decode)
//   out         the output bytes
constexpr uint32_t kSvcMaxStrings = 1024;     // strings per request
constexpr uint32_t kSvcInCap = 65536;         // input bytes per request
constexpr uint32_t kSvcHdrBytes = 256;
constexpr uint32_t kSvcOffBytes = 4352;       // (kSvcMaxStrings + 1) u32, 256-aligned
constexpr uint32_t kSvcInOffAt = kSvcHdrBytes;
constexpr uint32_t kSvcInAt = kSvcInOffAt + kSvcOffBytes;
constexpr uint32_t kSvcOutOffAt = kSvcInAt + kSvcInCap + 256;
constexpr uint32_t kSvcStatusAt = kSvcOutOffAt + kSvcOffBytes;
constexpr uint32_t kSvcOutAt = kSvcStatusAt + kSvcMaxStrings + 256;
// the encode bound of a full request (qhuff_encode_bound: 30-bit codes, 7
// bytes of framing per literal, 16 slack), rounded up
constexpr uint32_t kSvcOutCap =
    ((kSvcInCap * 30 + 7) / 8 + 7 * kSvcMaxStrings + 16 + 4095) & ~4095u;
constexpr uint32_t kSvcSlotBytes = (kSvcOutAt + kSvcOutCap + 4095) & ~4095u;
// device scratch per slot (a request of more than one tile): the slot's
// layout; in_off and in are copied in, the tile loop reads them and writes
// out_off, status and out at device-memory latency, and those are copied
// back into the slot at the end
constexpr uint32_t kSvcScratchBytes = kSvcSlotBytes;
static_assert(kSvcInOffAt % 256 == 0 && kSvcInAt % 256 == 0
              && kSvcOutOffAt % 256 == 0 && kSvcStatusAt % 256 == 0
              && kSvcOutAt % 256 == 0, "slot regions 256-aligned");

// a piece coded straight from its slot: one staged tile (64 strings, the
// stage's bytes; qhuff_service.hip checks it against kStageCap)
constexpr uint32_t kSvcTileBytes = 3072;

constexpr uint32_t kSvcOpDecode = 0;
constexpr uint32_t kSvcOpEncode = 1;

struct SvcHdr
{
    // the request's first 16 bytes are read by one 16-byte load per poll:
    // the host writes n, in_bytes and opmode, then req (release), all in one
    // cache line, so a load that sees the new req sees the fields too
    uint32_t req;                // host: sequence of the posted request (last)
    uint32_t n;                  // strings
    uint32_t in_bytes;
    uint32_t opmode;             // kSvcOp* | encode mode << 8
    uint32_t pad0[28];           // (the device's words on their own line)
    uint32_t done;               // device: sequence of the last served request
    uint32_t total;              // device: its output bytes
    uint32_t pad1[30];
};
static_assert(sizeof(SvcHdr) <= kSvcHdrBytes, "slot header");

struct SvcArgs
{
    uint8_t *slots;              // device view of the pinned slots
    uint8_t *scratch;            // device memory, kSvcScratchBytes per slot
    const uint32_t *ctl;         // device view of the pinned control word
                                 // [0]: stop
    uint64_t *active;            // device: last time any wave served (100 MHz)
    const uint32_t *win;
    const uint16_t *sorted;
    const uint16_t *long2;
    const uint2 *enc;
    uint64_t idle_ticks;         // a wave leaves after this long with no
                                 // request served by any wave (100 MHz ticks)
    uint64_t life_ticks;         // and after this long in any case
};

template <class T>
__device__ __forceinline__ const QH_GLB T *
glb(const T *p)
{
    return (const QH_GLB T *) p;
}

template <class T>
__device__ __forceinline__ QH_GLB T *
glb(T *p)
{
    return (QH_GLB T *) p;
}

// ev0 / ev1 non-null: the launch records its own start / stop time in them
// (hipExtLaunchKernelGGL: the dispatch's timestamps, no extra queue packets)
// full: the kernel variant with big-tile slots and cooperative long strings
// (qhuff_pipeline.h); the lean one is the default (qhuff_host.cpp)
hipError_t launch_encode(const EncArgs &a, uint32_t grid, hipStream_t st,
                         hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                         bool full = false);
// keep: the kernel that keeps a rejected string's bytes decoded before its
// error (qhuff_shim.cpp)
hipError_t launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st,
                         hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                         bool keep = false, bool full = false);
hipError_t launch_hash(const HashArgs &a, uint32_t max_grid, hipStream_t st,
                       hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
hipError_t hash_occupancy(int *blocks_per_cu);
// off[0 .. n) += add (shard stitching, qhuff_*_batch_multi)
hipError_t launch_rebase(uint32_t *off, uint64_t n, uint32_t add,
                         hipStream_t st);
int hash_waves_per_block();
hipError_t encode_occupancy(int *blocks_per_cu);
hipError_t decode_occupancy(int *blocks_per_cu);
size_t encode_lds_bytes();
size_t decode_lds_bytes();
int encode_waves_per_block();
int decode_waves_per_block();
uint32_t decode_tile_strings();            // strings per decode tile
hipError_t launch_service(const SvcArgs &a, uint32_t grid, hipStream_t st);
bool ctx_has_service(const qhuff_ctx *c);   // (qhuff_host.cpp)
int decode_keep_rejected(qhuff_ctx *c, const uint8_t *in,
                         const uint32_t *in_off, uint32_t n, uint8_t *out,
                         uint32_t *out_off, uint8_t *status);
int service_waves_per_block();
size_t service_lds_bytes();

}  // namespace qhuff
