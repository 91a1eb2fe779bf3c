// qhuff_fastwalk.h -- where the reference's complete-string decoder stops.
//
// huff_decode_fast (lsqpack.c:5243-5466) decodes through a 64-bit bit buffer
// and a 16-bit window table (hdecs[], at most three whole codes per window,
// lsqpack.c:5222-5229).  Its result for a valid string depends only on the
// code lengths of the decoded symbols and on dst_len: where the refills
// fall, which window reaches a code longer than 16 bits (slow_path) or
// produces more symbols than dst has room for (dst_ended), and the back-off
// to the previous byte-aligned symbol boundary.  walk() replays exactly that
// control flow over the lengths the GPU already decoded; no bit is decoded
// here.  Plain C++ (host code, also compiled by tests/c/ on the CPU).
#pragma once

#include <stdint.h>

namespace qhuff {

enum FastEnd : uint8_t
{
    kFastDone = 0,      // reached the end of input (the OK path)
    kFastDstEnded = 1,  // END_DST (lsqpack.c:5438-5450)
    kFastSlow = 2,      // slow_path: nibble decoder from n_src (5452-5465)
};

struct FastStop
{
    FastEnd end;
    uint32_t n_dst;     // symbols written (after the back-off, if any)
    uint32_t n_src;     // source bytes consumed
};

// symbols of the window at symbol i: up to three whole codes within `bits`
inline unsigned
fast_window(const uint8_t *len, uint32_t n, uint32_t i, unsigned bits,
            unsigned *used)
{
    unsigned k = 0, b = 0;
    while (k < 3 && i + k < n && b + len[i + k] <= bits)
        b += len[i + k++];
    *used = b;
    return k;
}

// len[0..n): code lengths of a valid string's symbols, src_len its encoded
// length (the bits after the last symbol are EOS padding, < 8).
inline FastStop
fast_walk(const uint8_t *len, uint32_t n, uint32_t src_len, uint32_t dst_len)
{
    uint32_t R = 0;          // source bytes shifted into the buffer
    unsigned avail = 0;      // bits in the buffer
    uint32_t d = 0;          // symbols written
    FastEnd end = kFastDone;
    for (;;)
    {
        // refill with whole bytes while at most 56 bits are held
        // (lsqpack.c:5267-5309: 6-8 bytes at once, or one at a time)
        if (R >= src_len)
            break;
        while (R < src_len && avail <= 56)
        {
            ++R;
            avail += 8;
        }
        if (dst_len - d >= 64 / 5 && avail >= 16)
        {
            // unchecked loop (lsqpack.c:5311-5328)
            unsigned k, used;
            do
            {
                k = fast_window(len, n, d, 16, &used);
                d += k;
                avail -= used;
            } while (avail >= 16 && k);
            if (avail < 16)
                continue;
            end = kFastSlow;
            goto back_off;
        }
        while (avail >= 16)
        {
            // checked loop (lsqpack.c:5330-5359)
            unsigned used;
            const unsigned k = fast_window(len, n, d, 16, &used);
            if (k && d + k <= dst_len)
            {
                d += k;
                avail -= used;
            }
            else
            {
                end = d + k > dst_len ? kFastDstEnded : kFastSlow;
                goto back_off;
            }
        }
    }
    // the last window, padded with ones (lsqpack.c:5362-5407); a valid
    // string's remaining symbols are whole within `avail` bits
    if (avail >= 5 && d < n)
    {
        unsigned used;
        const unsigned k = fast_window(len, n, d, avail, &used);
        if (d + k > dst_len)
        {
            end = kFastDstEnded;
            goto back_off;
        }
        d += k;
    }
    return FastStop{kFastDone, d, src_len};
back_off:
    // previous byte boundary (lsqpack.c:5442-5445, 5454-5457)
    while ((avail & 7) && d > 0)
        avail += len[--d];
    return FastStop{end, d, R - (avail >> 3)};
}

}  // namespace qhuff
