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

#include "qhuff_tables.h"

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

// Canonical first code and count of every code length (RFC 7541 Appendix B,
// kLen), for code_completes().
struct CanonLens
{
    uint32_t first[31], count[31];
};

constexpr CanonLens
make_canon_lens()
{
    CanonLens c{};
    for (int s = 0; s < 257; ++s)
        c.count[kLen[s]]++;
    uint32_t next = 0;
    for (int L = 1; L <= 30; ++L)
    {
        next <<= 1;
        c.first[L] = next;
        next += c.count[L];
    }
    return c;
}

constexpr CanonLens kCanonLens = make_canon_lens();

// whether the left-aligned bits of w start with a whole code of at most
// maxbits bits (the question hdecs[] answers for a window, lsqpack.c:5371)
inline bool
code_completes(uint32_t w, unsigned maxbits)
{
    for (unsigned L = 1; L <= maxbits && L <= 30; ++L)
        if (kCanonLens.count[L]
            && (w >> (32 - L)) - kCanonLens.first[L] < kCanonLens.count[L])
            return true;
    return false;
}

// bits [pos, pos + 32) of src (big-endian bit order), ones past src_len
inline uint32_t
bits_at(const uint8_t *src, uint32_t src_len, uint32_t pos)
{
    uint32_t w = 0;
    for (unsigned k = 0; k < 32; ++k)
    {
        const uint32_t b = pos + k;
        const uint32_t bit = b < 8 * src_len ? (src[b >> 3] >> (7 - (b & 7))) & 1
                                             : 1u;
        w = (w << 1) | bit;
    }
    return w;
}

// The same replay for an INVALID string (the GPU rejected it): len[0..n)
// are the code lengths of the symbols decoded before the error, followed,
// when the error is the EOS code in the data, by a 30 for the EOS code
// itself -- no window of the fast decoder holds it, so the walk takes the
// slow path there, as the reference does (its nibble decoder then finds the
// EOS, lsqpack.c:3480-3497).  Otherwise the error is the padding, found
// only after the last window (lsqpack.c:5362-5426): end kFastDone means the
// reference returns ERROR; kFastDstEnded / kFastSlow as in fast_walk.  In
// that last window the reference's table decodes, after the string's last
// whole codes, one more code if the padded bits complete one within the
// window -- a code running past the input: ERROR before any room check
// (lsqpack.c:5373-5378); otherwise its symbols are written, or do not fit
// (END_DST, 5398-5399).
inline FastStop
fast_walk_invalid(const uint8_t *len, uint32_t n, const uint8_t *src,
                  uint32_t src_len, uint32_t dst_len)
{
    uint32_t R = 0;
    unsigned avail = 0;
    uint32_t d = 0;
    FastEnd end = kFastDone;
    for (;;)
    {
        if (R >= src_len)
            break;
        while (R < src_len && avail <= 56)
        {
            ++R;
            avail += 8;
        }
        if (dst_len - d >= 64 / 5 && avail >= 16)
        {
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
    if (avail >= 5)
    {
        unsigned used;
        const unsigned k = fast_window(len, n, d, avail, &used);
        if (k < 3 && code_completes(bits_at(src, src_len, 8 * R - avail + used),
                                    16 - used))
            return FastStop{kFastDone, 0, 0};            // ERROR
        if (k && d + k > dst_len)
        {
            end = kFastDstEnded;
            goto back_off;
        }
    }
    return FastStop{kFastDone, 0, 0};                    // ERROR (padding)
back_off:
    while ((avail & 7) && d > 0)
        avail += len[--d];
    return FastStop{end, d, R - (avail >> 3)};
}

}  // namespace qhuff
