// C entry to qhuff_fastwalk.h for tests/test_fastwalk.py (CPU, no GPU).
#include "../../ls-qpack_amd/csrc/qhuff_fastwalk.h"

extern "C" void
qh_fast_walk(const uint8_t *len, uint32_t n, uint32_t src_len,
             uint32_t dst_len, uint32_t out[3])
{
    const qhuff::FastStop f = qhuff::fast_walk(len, n, src_len, dst_len);
    out[0] = f.end;
    out[1] = f.n_dst;
    out[2] = f.n_src;
}

extern "C" void
qh_fast_walk_invalid(const uint8_t *len, uint32_t n, const uint8_t *src,
                     uint32_t src_len, uint32_t dst_len, uint32_t out[3])
{
    const qhuff::FastStop f = qhuff::fast_walk_invalid(len, n, src, src_len,
                                                       dst_len);
    out[0] = f.end;
    out[1] = f.n_dst;
    out[2] = f.n_src;
}
