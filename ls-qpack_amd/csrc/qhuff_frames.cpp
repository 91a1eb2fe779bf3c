// qhuff_frames.cpp -- literal-span pre-parse of QPACK wire data and the
// batched literal decode built on it.
//
// The reference decodes string literals one at a time from inside its
// resumable instruction readers:
//   encoder stream   lsqpack_dec_enc_in       lsqpack.c:4574-4960
//   field section    parse_header_data et al. lsqpack.c:3567-3915
// and every Huffman literal goes through lsqpack_huff_decode
// (lsqpack.c:3718, 3795, 4714, 4824, 4908).  Here a cheap host pass walks
// the instruction framing only (prefixed integers, RFC 9204 sections 4.3 and
// 4.5 / lsqpack_dec_int(24), lsqpack.c:2372-2460) and records each literal's
// span; the Huffman spans of any number of blocks are then gathered into one
// pinned batch and decoded by the GPU kernel in a single launch.  Dynamic
// table references, blocked streams and the decoder's state machine stay
// with the reference: the scan resolves no index and allocates nothing.
// Plain C++ (no HIP): tests/c/ also builds it with ASan/UBSan on the CPU.
#include <stdint.h>
#include <string.h>

#include "../../include/qhuff.h"

namespace {

// lsqpack_dec_int (lsqpack.c:2372-2437) on a complete buffer: 0 ok, -1 the
// buffer ends inside the integer, -2 the value does not fit 64 bits.  The
// reference's other -2 (out of input after >= LSQPACK_UINT64_ENC_SZ = 11
// bytes, lsqpack.c:2413-2423) counts bytes across resumed calls; in one call
// the loop reads at most the prefix byte and 10 continuation bytes and
// checks for input before the 10th, so out of input is always -1 here.
int
dec_int(const uint8_t **pp, const uint8_t *end, unsigned prefix_bits,
        uint64_t *v_out)
{
    const uint8_t *p = *pp;
    if (p >= end)
        return -1;
    const unsigned pmax = (1u << prefix_bits) - 1;
    uint64_t v = *p++ & pmax;
    if (v < pmax)
    {
        *pp = p;
        *v_out = v;
        return 0;
    }
    unsigned M = 0;
    uint8_t B;
    do
    {
        if (p >= end)
            return -1;
        B = *p++;
        v += (uint64_t) (B & 0x7f) << M;
        M += 7;
    } while ((B & 0x80) && M < 64);
    if (M <= 63 || (M == 70 && p[-1] <= 1 && (v & (1ull << 63))))
    {
        *pp = p;
        *v_out = v;
        return 0;
    }
    return -2;
}

// lsqpack_dec_int24 (lsqpack.c:2443-2460): values >= 2^24 are errors
int
dec_int24(const uint8_t **pp, const uint8_t *end, unsigned prefix_bits,
          uint32_t *v_out)
{
    uint64_t v;
    const int r = dec_int(pp, end, prefix_bits, &v);
    if (r)
        return r;
    if (v >= (1u << 24))
        return -2;
    *v_out = (uint32_t) v;
    return 0;
}

struct Sink
{
    const uint8_t *base;
    uint32_t pos_base;
    qhuff_literal *lits;
    uint32_t cap, n;
    bool overflow;
};

// a string literal whose H bit sits just above its N-bit length prefix
// (the layouts lsqpack_enc_enc_str writes for N = 3, 5, 7, lsqpack.c:839).
// max_len > 0: a declared length above it is an error as soon as the length
// is decoded, before the payload is looked for -- the field-section rule
// (LSXPACK_MAX_STRLEN, lsqpack.c:3682-3685 values, 3769-3772 names; pinned
// by test/test_header_alloc_clamp.c:108-135).
int
literal(Sink &s, const uint8_t **pp, const uint8_t *end, unsigned prefix_bits,
        unsigned kind, uint32_t instr, uint32_t max_len)
{
    const uint8_t *p = *pp;
    if (p >= end)
        return -1;
    const uint8_t *const start = p;
    const unsigned h = (*p >> prefix_bits) & 1;
    uint32_t len;
    const int r = dec_int24(&p, end, prefix_bits, &len);
    if (r)
        return r;
    if (max_len && len > max_len)
        return -2;
    if ((uint64_t) (end - p) < len)
        return -1;
    if (s.n < s.cap)
    {
        qhuff_literal &l = s.lits[s.n];
        l.pos = s.pos_base + (uint32_t) (p - s.base);
        l.len = len;
        l.huffman = (uint8_t) h;
        l.prefix_bits = (uint8_t) prefix_bits;
        l.kind = (uint8_t) kind;
        l.hdr_len = (uint8_t) (p - start);
        l.instr = s.pos_base + instr;
    }
    else
        s.overflow = true;
    ++s.n;
    *pp = p + len;
    return 0;
}

int
rc_of(int r)
{
    return r == -1 ? QHUFF_ETRUNC : QHUFF_EPROTO;
}

}  // namespace

// Name lengths of the QPACK static table (RFC 9204 Appendix A; the
// reference's static_table[], lsqpack.c:104-209 -- the list in
// tests/golden/qpack_static_table.json, which test_frames.py checks this
// against through qhuff_decode_literals_ex).
static const uint8_t kStaticNameLen[99] = {
    10, 5, 3, 19, 14, 6, 4, 4, 17, 13, 13, 4, 8, 7, 10, 7, 7, 7, 7, 7, 7, 7,
    7, 7, 7, 7, 7, 7, 7, 6, 6, 15, 13, 28, 28, 27, 13, 13, 13, 13, 13, 13,
    16, 16, 12, 12, 12, 12, 12, 12, 12, 12, 12, 12, 12, 5, 25, 25, 25, 4, 4,
    22, 16, 7, 7, 7, 7, 7, 7, 7, 7, 7, 15, 32, 32, 28, 28, 28, 28, 29, 30,
    29, 29, 7, 13, 23, 10, 9, 9, 8, 6, 7, 6, 19, 25, 10, 15, 15, 15};

namespace qhuff {

// The length of the name a field-section VALUE literal's instruction refers
// to, when the framing alone knows it: a static name reference (01NT with
// T = 1, 4-bit index; lsqpack.c:3620-3642 header_out_begin_static_nameref
// copies static_table[idx].name into the header buffer) -> its length;
// a dynamic or post-base reference (the dynamic table stays with the
// reference) or anything else -> 0.  buf: the buffer lits' offsets are
// relative to (the instruction lies in [l.instr, l.pos - l.hdr_len)).
uint32_t
field_ref_name_len(const uint8_t *buf, const struct qhuff_literal &l)
{
    if (l.kind != QHUFF_LIT_VALUE || l.hdr_len > l.pos
            || (uint64_t) l.instr + 1 > l.pos - l.hdr_len)
        return 0;
    const uint8_t *p = buf + l.instr, *const end = buf + (l.pos - l.hdr_len);
    if ((*p & 0xd0) != 0x50)                 // 01NT, T = 1
        return 0;
    uint32_t idx;
    if (dec_int24(&p, end, 4, &idx) || idx >= sizeof(kStaticNameLen))
        return 0;
    return kStaticNameLen[idx];
}

}  // namespace qhuff

// (ABI 7) the scanners' integer decoder on its own: lsqpack_dec_int
// (lsqpack.c:2372-2437) on a complete buffer -- pinned to the reference's
// own vectors (test/test_int.c:19-183, tests/golden/kat_int.json)
extern "C" int
qhuff_dec_int(const uint8_t *buf, size_t len, unsigned prefix_bits,
              uint64_t *value, size_t *consumed)
{
    if ((!buf && len) || !value || !consumed || prefix_bits < 1
            || prefix_bits > 8)
        return QHUFF_EINVAL;
    const uint8_t *p = buf;
    uint64_t v = 0;
    const int r = dec_int(&p, buf + len, prefix_bits, &v);
    if (r)
        return rc_of(r);
    *value = v;
    *consumed = (size_t) (p - buf);
    return QHUFF_OK;
}

extern "C" int
qhuff_scan_field_section(const uint8_t *buf, size_t len, uint32_t pos_base,
                         struct qhuff_literal *lits, uint32_t max_lits,
                         uint32_t *n_lits)
{
    if ((!buf && len) || (!lits && max_lits) || !n_lits
            || (uint64_t) pos_base + len > 0xffffffffu)
        return QHUFF_EINVAL;
    *n_lits = 0;
    Sink s{buf, pos_base, lits, max_lits, 0, false};
    const uint8_t *p = buf, *const end = buf + len;
    const uint32_t max_str = QHUFF_MAX_STRLEN;
    uint64_t v;
    int r;
    // section prefix: Required Insert Count (8-bit prefix), S + Delta Base
    // (7-bit prefix) -- RFC 9204 4.5.1, parse_header_prefix, lsqpack.c:3955-4046
    if ((r = dec_int(&p, end, 8, &v)) || (r = dec_int(&p, end, 7, &v)))
        return rc_of(r);
    while (p < end)
    {
        const uint8_t b = *p;
        const uint32_t at = (uint32_t) (p - buf);
        uint32_t idx;
        if (b & 0x80)                          // 1Txxxxxx indexed field line
            r = dec_int24(&p, end, 6, &idx);
        else if (b & 0x40)                     // 01NTxxxx literal, name ref
        {
            r = dec_int24(&p, end, 4, &idx);
            if (!r)
                r = literal(s, &p, end, 7, QHUFF_LIT_VALUE, at, max_str);
        }
        else if (b & 0x20)                     // 001NHxxx literal name
        {
            r = literal(s, &p, end, 3, QHUFF_LIT_NAME, at, max_str);
            if (!r)
                r = literal(s, &p, end, 7, QHUFF_LIT_VALUE, at, max_str);
        }
        else if (b & 0x10)                     // 0001xxxx indexed post-base
            r = dec_int24(&p, end, 4, &idx);
        else                                   // 0000Nxxx post-base name ref
        {
            r = dec_int24(&p, end, 3, &idx);
            if (!r)
                r = literal(s, &p, end, 7, QHUFF_LIT_VALUE, at, max_str);
        }
        if (r)
            return rc_of(r);
    }
    *n_lits = s.n;
    return s.overflow ? QHUFF_ERANGE : QHUFF_OK;
}

extern "C" int
qhuff_scan_encoder_stream(const uint8_t *buf, size_t len, uint32_t pos_base,
                          struct qhuff_literal *lits, uint32_t max_lits,
                          uint32_t *n_lits, size_t *consumed)
{
    if ((!buf && len) || (!lits && max_lits) || !n_lits || !consumed
            || (uint64_t) pos_base + len > 0xffffffffu)
        return QHUFF_EINVAL;
    *n_lits = 0;
    *consumed = 0;
    Sink s{buf, pos_base, lits, max_lits, 0, false};
    const uint8_t *p = buf, *const end = buf + len;
    while (p < end)
    {
        const uint8_t *q = p;
        const uint8_t b = *q;
        const uint32_t at = (uint32_t) (p - buf);
        const uint32_t n0 = s.n;
        uint32_t v;
        int r;
        if (b & 0x80)                // 1Txxxxxx insert with name reference
        {
            r = dec_int24(&q, end, 6, &v);
            if (!r)
                r = literal(s, &q, end, 7, QHUFF_LIT_VALUE, at, 0);
        }
        else if (b & 0x40)           // 01Hxxxxx insert with literal name
        {
            r = literal(s, &q, end, 5, QHUFF_LIT_NAME, at, 0);
            if (!r)
                r = literal(s, &q, end, 7, QHUFF_LIT_VALUE, at, 0);
        }
        else                         // 001xxxxx capacity / 000xxxxx dup
        {
            uint64_t w;
            r = dec_int(&q, end, 5, &w);
            if (!r && !(b & 0x20) && w >= (1u << 24))
                r = -2;
        }
        if (r == -1)
        {
            // a partial instruction: stop before it (the reference resumes
            // there when more stream data arrives, lsqpack.c:4574)
            s.n = n0;
            break;
        }
        if (r)
            return QHUFF_EPROTO;
        p = q;
    }
    if (s.n > s.cap)
    {
        *n_lits = s.n;
        return QHUFF_ERANGE;
    }
    *n_lits = s.n;
    *consumed = (size_t) (p - buf);
    return QHUFF_OK;
}

// ---- literal framing from a precomputed payload ---
//
// lsqpack_enc_enc_str (lsqpack.c:839-876) with its Huffman step already done
// by a PAYLOAD-mode batch: the strict size test (lsqpack.c:848), the H bit
// and the prefixed length (lsqpack_val2len / lsqpack_enc_int_nocheck,
// lsqpack.c:767-836), the payload or the raw string, -1 when dst_len is
// short.  dst[0] bits above the H bit are kept, as in the reference.

namespace {

unsigned
val2len(uint64_t v, unsigned prefix_bits)
{
    const uint64_t mask = (1ull << prefix_bits) - 1;
    unsigned n = 1;
    if (v >= mask)
        for (v -= mask, ++n; v >= 128; v >>= 7)
            ++n;
    return n;
}

void
put_int(uint8_t *dst, uint64_t v, unsigned prefix_bits)
{
    const uint64_t mask = (1ull << prefix_bits) - 1;
    if (v < mask)
    {
        *dst |= (uint8_t) v;
        return;
    }
    *dst++ |= (uint8_t) mask;
    for (v -= mask; v >= 128; v >>= 7)
        *dst++ = (uint8_t) (0x80 | v);
    *dst = (uint8_t) v;
}

}  // namespace

extern "C" int
qhuff_frame_literal(unsigned prefix_bits, unsigned char *dst, size_t dst_len,
                    const unsigned char *str, unsigned str_len,
                    const unsigned char *huff, unsigned huff_len)
{
    if (!dst || (!str && str_len) || (!huff && huff_len)
            || (prefix_bits != 3 && prefix_bits != 5 && prefix_bits != 7))
        return -1;
    const bool h = huff_len < str_len;
    const unsigned n = h ? huff_len : str_len;
    const unsigned len_size = val2len(n, prefix_bits);
    if ((uint64_t) len_size + n > dst_len)
        return -1;
    dst[0] &= (uint8_t) ~((1u << (prefix_bits + 1)) - 1);
    if (h)
        dst[0] |= (uint8_t) (1u << prefix_bits);
    put_int(dst, n, prefix_bits);
    memcpy(dst + len_size, h ? huff : str, n);
    return (int) (len_size + n);
}
