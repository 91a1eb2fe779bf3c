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

hipError_t launch_encode(const EncArgs &a, uint32_t grid, hipStream_t st);
hipError_t launch_decode(const DecArgs &a, uint32_t grid, hipStream_t st);
hipError_t launch_hash(const HashArgs &a, uint32_t max_grid, hipStream_t st);
hipError_t hash_occupancy(int *blocks_per_cu);
hipError_t encode_occupancy(int *blocks_per_cu);
hipError_t decode_occupancy(int *blocks_per_cu);
size_t encode_lds_bytes();
size_t decode_lds_bytes();
int encode_waves_per_block();
int decode_waves_per_block();
uint32_t decode_tile_strings();            // strings per decode tile

}  // namespace qhuff
