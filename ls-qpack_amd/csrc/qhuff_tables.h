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
#pragma once
#include <stdint.h>

namespace qhuff {

constexpr int kWinBits = 12;
constexpr int kWinSize = 1 << kWinBits;
constexpr int kMaxLong = 16;            // lengths 13..30 that occur (14 used)

// window entry: sym0 [7:0] | sym1 [15:8] | bits consumed by all nsym
//               symbols c [19:16] | len0 [23:20] | nsym [25:24] |
//               32 - c [31:26] (the decoder's alignbit shift); nsym == 0:
//               the first code is longer than 12 bits (entry < 1 << 24)
struct LongLen { uint32_t len, first, count, base; };

struct HostTables
{
    uint32_t code[257];
    uint8_t bits[257];
    uint32_t win[kWinSize];
    LongLen longc[kMaxLong];
    uint32_t n_long;
    uint16_t sorted[257];
};

void build_tables(HostTables *t);

}  // namespace qhuff
