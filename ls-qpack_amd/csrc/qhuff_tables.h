// qhuff_tables.h -- static RFC 7541 Huffman tables, built on the host at
// context open and uploaded once.
//
// The reference keeps four tables in huff-tables.h (lsqpack.c:72; missing from
// the reference mount).  This codec needs different layouts, shaped for LDS
// and for one-string-per-lane kernels, so it derives its own from the 257 RFC
// 7541 Appendix B code lengths:
//
//   enc[257]      {code (right-aligned), bits}      -- encoder (lsqpack.c:5144)
//   win[4096]     12-bit window -> up to 2 symbols   -- decoder fast step
//                 (the 16-bit hdecs[] of lsqpack.c:5317 does not fit LDS next
//                 to the other stages; 12 bits covers every code of 5..12
//                 bits, i.e. all printable ASCII but a handful)
//   longc[]       canonical (first code, count, base) for lengths 13..30 --
//                 decoder step for long codes (the reference switches to its
//                 nibble FSM there, lsqpack.c:5452-5465)
//   sorted[257]   symbols in canonical order (index -> symbol)
//   long2[640]    long codes by leading ones + 5 bits (decoder long step)
#pragma once
#include <stdint.h>

namespace qhuff {

// decode window width (QH_WIN_BITS): 13 bits = 32 KB of LDS table, one more
// two-symbol pair (6 + 7 bits) per lookup than 12
#ifndef QH_WIN_BITS
#define QH_WIN_BITS 13
#endif
constexpr int kWinBits = QH_WIN_BITS;
constexpr int kWinSize = 1 << kWinBits;
constexpr int kMaxLong = 16;            // lengths 13..30 that occur (14 used)

// window entry: sym0 [7:0] | bits consumed by all nsym symbols c [11:8] |
//               len0 [15:12] | sym1 [23:16] | nsym [25:24] |
//               32 - c [31:26] (the decoder's alignbit shift); nsym == 0:
//               the first code is longer than the window (entry < 1 << 24).
//               sym1 sits at [23:16] so the decoder stores it with
//               ds_write_b8_d16_hi, no shift.
struct LongLen { uint32_t len, first, count, base; };

// RFC 7541 Appendix B code lengths, symbols 0..256 (EOS = 256).
constexpr uint8_t kLen[257] = {
    13,23,28,28,28,28,28,28,28,24,30,28,28,30,28,28,28,28,28,28,28,28,30,28,28,28,28,28,28,28,28,28,
     6,10,10,12,13, 6, 8,11,10,10, 8,11, 8, 6, 6, 6, 5, 5, 5, 6, 6, 6, 6, 6, 6, 6, 7, 8,15, 6,12,10,
    13, 6, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 8, 7, 8,13,19,13,14, 6,
    15, 5, 6, 5, 6, 5, 6, 6, 6, 5, 7, 7, 6, 6, 6, 5, 6, 7, 6, 5, 5, 6, 7, 7, 7, 7, 7,15,11,14,13,28,
    20,22,20,20,22,22,22,23,22,23,23,23,23,23,24,23,24,24,22,23,24,23,23,23,23,21,22,23,22,23,23,24,
    22,21,20,22,22,23,23,21,23,22,22,24,21,22,23,23,21,21,22,21,23,22,23,23,20,22,22,22,23,22,22,23,
    26,26,20,19,22,23,22,25,26,26,26,27,27,26,24,25,19,21,26,27,27,26,27,24,21,21,26,26,28,27,27,27,
    20,24,20,21,22,21,21,23,22,22,25,25,24,24,26,23,26,27,26,26,27,27,27,27,27,28,27,27,27,27,27,26,
    30,
};

// Canonical parameters of the code lengths above the window (13..30),
// computed at compile time: the code is static (RFC 7541 Appendix B), so the
// decoder's long-code step compares against immediates.
struct LongTab
{
    uint32_t n;
    LongLen l[kMaxLong];
};

constexpr LongTab
make_long_tab()
{
    LongTab t{};
    uint32_t count[31] = {};
    for (int s = 0; s < 257; ++s)
        count[kLen[s]]++;
    uint32_t next = 0, idx = 0;
    for (int L = 1; L <= 30; ++L)
    {
        next <<= 1;
        if (L > kWinBits && count[L])
            t.l[t.n++] = LongLen{(uint32_t) L, next, count[L], idx};
        next += count[L];
        idx += count[L];
    }
    return t;
}

constexpr LongTab kLongTab = make_long_tab();

// Long codes (14..30 bits) by their leading ones: every such code starts
// with n1 >= 12 ones, and after its first zero has at most 5 more bits
// (RFC 7541 Appendix B).  long2[(min(n1, 31) - 12) * 32 + the 5 bits after
// the first zero] = sym | (L - 14) << 9 (0xffff: no code of 14..30 bits
// there); n1 >= 30 is the EOS code (sym 256, L 30).  The decoder's in-loop
// long step: a count of leading ones and one lookup.
constexpr int kLong2N1 = 12;
constexpr int kLong2Rows = 32 - kLong2N1;
constexpr int kLong2Size = kLong2Rows * 32;

struct HostTables
{
    uint32_t code[257];
    uint8_t bits[257];
    uint32_t win[kWinSize];
    LongLen longc[kMaxLong];
    uint32_t n_long;
    uint16_t sorted[257];
    uint16_t long2[kLong2Size];
};

void build_tables(HostTables *t);

}  // namespace qhuff
