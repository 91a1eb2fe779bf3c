// qhuff_tables.cpp -- derive every table the kernels use from the RFC 7541
// Appendix B code lengths (canonical Huffman: codes assigned in (length,
// symbol) order).  Host code, run once per context.
#include "qhuff_tables.h"

#include <string.h>

namespace qhuff {

namespace {

struct Canon
{
    uint32_t first[31], count[31], base[31];
    uint16_t sorted[257];
};

void
canon_build(Canon *c, uint32_t *code)
{
    memset(c, 0, sizeof(*c));
    for (int s = 0; s < 257; ++s)
        c->count[kLen[s]]++;
    uint32_t next = 0, idx = 0;
    for (int L = 1; L <= 30; ++L)
    {
        next <<= 1;
        c->first[L] = next;
        c->base[L] = idx;
        next += c->count[L];
        idx += c->count[L];
    }
    uint32_t fill[31];
    for (int L = 1; L <= 30; ++L)
        fill[L] = 0;
    for (int s = 0; s < 257; ++s)          // symbol order within a length
    {
        int L = kLen[s];
        code[s] = c->first[L] + fill[L];
        c->sorted[c->base[L] + fill[L]] = (uint16_t) s;
        fill[L]++;
    }
}

// Decode one symbol from the top `avail` bits of `w` (left-aligned in 32
// bits).  Returns the symbol and sets *len, or -1 if no code of length
// <= avail is complete.
int
canon_decode(const Canon *c, uint32_t w, int avail, int *len)
{
    for (int L = 1; L <= avail && L <= 30; ++L)
    {
        uint32_t v = w >> (32 - L);
        if (c->count[L] && v - c->first[L] < c->count[L])
        {
            *len = L;
            return c->sorted[c->base[L] + (v - c->first[L])];
        }
    }
    return -1;
}

}  // namespace

void
build_tables(HostTables *t)
{
    Canon c;
    canon_build(&c, t->code);
    for (int s = 0; s < 257; ++s)
        t->bits[s] = kLen[s];
    memcpy(t->sorted, c.sorted, sizeof(t->sorted));

    for (uint32_t w = 0; w < (uint32_t) kWinSize; ++w)
    {
        uint32_t left = w << (32 - kWinBits);
        int l0, l1;
        int s0 = canon_decode(&c, left, kWinBits, &l0);
        uint32_t e = 0;
        if (s0 >= 0 && s0 < 256)
        {
            e = (uint32_t) s0 | ((uint32_t) l0 << 8) | ((uint32_t) l0 << 12)
              | (1u << 24) | ((uint32_t) (32 - l0) << 26);
            int s1 = canon_decode(&c, left << l0, kWinBits - l0, &l1);
            if (s1 >= 0 && s1 < 256)
                e = (uint32_t) s0 | ((uint32_t) s1 << 16)
                  | ((uint32_t) (l0 + l1) << 8) | ((uint32_t) l0 << 12)
                  | (2u << 24) | ((uint32_t) (32 - l0 - l1) << 26);
        }
        t->win[w] = e;
    }

    for (int r = 0; r < kLong2Rows; ++r)
        for (uint32_t x = 0; x < 32; ++x)
        {
            const int n1 = kLong2N1 + r;
            // n1 ones, a zero, then x's 5 bits (fewer when they run out)
            uint32_t w = n1 >= 32 ? 0xffffffffu : ~(0xffffffffu >> n1);
            if (n1 <= 26)
                w |= x << (26 - n1);
            else if (n1 < 31)
                w |= x >> (n1 - 26);
            int L;
            const int sym = canon_decode(&c, w, 30, &L);
            t->long2[r * 32 + x] = sym >= 0 && L > kWinBits
                ? (uint16_t) ((uint32_t) sym | ((uint32_t) (L - 14) << 9))
                : (uint16_t) 0xffff;
        }

    t->n_long = 0;
    for (int L = kWinBits + 1; L <= 30; ++L)
        if (c.count[L])
        {
            LongLen &ll = t->longc[t->n_long++];
            ll.len = (uint32_t) L;
            ll.first = c.first[L];
            ll.count = c.count[L];
            ll.base = c.base[L];
        }
}

}  // namespace qhuff
