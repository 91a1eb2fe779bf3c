// san_check.cpp -- the host code that parses untrusted wire bytes, run under
// AddressSanitizer + UndefinedBehaviorSanitizer on the CPU (SURVEY.md 5:
// "host ASan/UBSan").  TEST INFRASTRUCTURE: links the
// CPU oracle (oracle/qhuff_oracle.c) as the checker.
//
// Built by tests/test_sanitize.py with -fsanitize=address,undefined
// -fno-sanitize-recover=all (a report aborts), together with:
//   ls-qpack_amd/csrc/qhuff_frames.cpp   qhuff_scan_field_section,
//                                        qhuff_scan_encoder_stream,
//                                        qhuff_frame_literal
//   ls-qpack_amd/csrc/qhuff_fastwalk.h   the END_DST / slow-path replay
//   oracle/qhuff_oracle.c                lsqpack.c's Huffman functions
//
// Usage: san_check FILE...   every record of each file (u64 BE stream id,
// u32 BE size, payload; sizes clamped, bin/fuzz-decode.c:152-202) through
// BOTH scanners, then a seeded havoc of each record and of random bytes.
// For every literal the scanners report: its span lies in the record;
// Huffman payloads through oq_huff_decode at several dst_len, the fast-walk
// replay against it, and the streaming decoder fed in two chunks; decoded
// strings re-framed by qhuff_frame_literal (against oq_enc_enc_str) at
// exact and short dst_len.  Exit 0 only when every check holds.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/qhuff.h"
#include "../../ls-qpack_amd/csrc/qhuff_fastwalk.h"

extern "C" {
struct oq_retval { int status; unsigned n_dst, n_src; };
struct oq_dec_state { int resume; uint8_t state, eos; };
enum { OQ_OK, OQ_END_SRC, OQ_END_DST, OQ_ERROR };
void oq_init(void);
unsigned oq_enc_str_size(const unsigned char *str, unsigned len);
void oq_huffman_enc(const unsigned char *src, const unsigned char *end,
                    unsigned char *dst);
int oq_enc_enc_str(unsigned prefix_bits, unsigned char *dst, size_t dst_len,
                   const unsigned char *str, unsigned str_len);
struct oq_retval oq_huff_decode(const unsigned char *src, int src_len,
                                unsigned char *dst, int dst_len,
                                struct oq_dec_state *st, int final);
struct oq_retval oq_huff_decode_full(const unsigned char *src, int src_len,
                                     unsigned char *dst, int dst_len,
                                     struct oq_dec_state *st, int final);
void oq_code_of(unsigned sym, uint32_t *code, unsigned *bits);
}

static unsigned long n_checks, n_bad, n_lits, n_huff, n_records;
static uint8_t code_len[256];

static void
check(bool ok, const char *what, unsigned a, unsigned b)
{
    ++n_checks;
    if (!ok && n_bad++ < 20)
        fprintf(stderr, "FAIL %s (%u, %u)\n", what, a, b);
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t
rnd(void)
{
    uint64_t x = rng_state;
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return rng_state = x;
}

// exact-size heap copies, so ASan sees every byte past the end
static std::vector<uint8_t>
dup(const uint8_t *p, size_t n)
{
    return std::vector<uint8_t>(p, p + n);
}

static struct oq_retval
oracle_decode(const uint8_t *src, int sl, uint8_t *dst, int dl)
{
    struct oq_dec_state st = {0, 0, 0};
    return oq_huff_decode(src, sl, dst, dl, &st, 1);
}

static void
check_huffman(const uint8_t *src0, uint32_t sl)
{
    ++n_huff;
    std::vector<uint8_t> src = dup(src0, sl);
    const uint8_t *s = sl ? src.data() : nullptr;
    const uint32_t cap = sl * 8 / 5 + 1;
    uint8_t *full = (uint8_t *) malloc(cap);
    const struct oq_retval r = oracle_decode(s, (int) sl, full, (int) cap);
    check(r.status == OQ_OK || r.status == OQ_ERROR, "status", sl, r.status);
    if (r.status == OQ_OK)
    {
        check(r.n_src == sl && r.n_dst <= cap, "n_src", sl, r.n_dst);
        const uint32_t n = r.n_dst;
        // round trip through the encoder
        check(oq_enc_str_size(full, n) == sl, "size", sl, n);
        uint8_t *re = (uint8_t *) malloc(sl ? sl : 1);
        oq_huffman_enc(full, full + n, re);
        check(sl == 0 || memcmp(re, s, sl) == 0, "re-encode", sl, n);
        free(re);
        // the fast-walk replay vs the reference decoder at each dst_len
        std::vector<uint8_t> lens(n);
        bool has_long = false;
        for (uint32_t i = 0; i < n; ++i)
        {
            lens[i] = code_len[full[i]];
            has_long |= lens[i] > 16;
        }
        const uint32_t dls[] = {0, 1, n ? n - 1 : 0, n, n + 1, n + n / 2 + 2};
        for (uint32_t dl : dls)
        {
            uint8_t *d = (uint8_t *) malloc(dl ? dl : 1);
            const struct oq_retval w = oracle_decode(s, (int) sl, d, (int) dl);
            qhuff::FastStop f{qhuff::kFastDone, n, sl};
            if (n > dl || has_long)
                f = qhuff::fast_walk(lens.data(), n, sl, dl);
            struct oq_retval g;
            if (f.end == qhuff::kFastDone)
                g = {OQ_OK, f.n_dst, f.n_src};
            else if (f.end == qhuff::kFastDstEnded)
                g = {OQ_END_DST, f.n_dst, f.n_src};
            else
            {
                struct oq_dec_state st = {0, 0, 0};
                uint8_t *d2 = (uint8_t *) malloc(dl - f.n_dst ? dl - f.n_dst : 1);
                g = oq_huff_decode_full(s + f.n_src, (int) (sl - f.n_src), d2,
                                        (int) (dl - f.n_dst), &st, 1);
                if (g.status == OQ_OK || g.status == OQ_END_DST)
                {
                    g.n_dst += f.n_dst;
                    g.n_src += f.n_src;
                }
                free(d2);
            }
            check(g.status == w.status && g.n_dst == w.n_dst
                  && g.n_src == w.n_src, "fast_walk", sl, dl);
            free(d);
        }
        // re-framing (the encoder hook) at each prefix width
        for (unsigned p = 3; p <= 7; p += 2)
        {
            uint8_t want[16 + 2 * 4096], got[16 + 2 * 4096];
            if (n + 16 > sizeof want)
                break;
            want[0] = got[0] = 0xff;
            const int w = oq_enc_enc_str(p, want, sizeof want, full, n);
            std::vector<uint8_t> h = dup(s ? s : full, sl);
            const int g = qhuff_frame_literal(p, got, sizeof got, full, n,
                                              sl ? h.data() : nullptr, sl);
            check(w == g && (w < 0 || memcmp(want, got, w) == 0), "frame", p,
                  n);
            if (w > 0)
            {
                // exactly enough room, and one byte short, in exact buffers
                std::vector<uint8_t> ex((size_t) w), sh((size_t) w - 1 + 1);
                ex[0] = 0xff;
                check(qhuff_frame_literal(p, ex.data(), (size_t) w, full, n,
                                          sl ? h.data() : nullptr, sl) == w,
                      "frame exact", p, n);
                sh[0] = 0xff;
                check(qhuff_frame_literal(p, sh.data(), (size_t) w - 1, full,
                                          n, sl ? h.data() : nullptr, sl)
                          == -1, "frame short", p, n);
            }
        }
    }
    // the streaming decoder, input split in two (resumable state)
    if (sl)
    {
        const uint32_t cut = (uint32_t) (rnd() % (sl + 1));
        struct oq_dec_state st = {0, 0, 0};
        uint8_t *d = (uint8_t *) malloc(cap);
        struct oq_retval a = oq_huff_decode_full(s, (int) cut, d, (int) cap,
                                                 &st, cut == sl);
        if (cut < sl && (a.status == OQ_END_SRC || a.status == OQ_OK))
        {
            struct oq_retval b = oq_huff_decode_full(s + a.n_src,
                                                     (int) (sl - a.n_src),
                                                     d + a.n_dst,
                                                     (int) (cap - a.n_dst),
                                                     &st, 1);
            a.status = b.status;
            if (b.status == OQ_OK)
                a.n_dst += b.n_dst;
        }
        check(a.status == r.status, "streaming status", sl, cut);
        if (a.status == OQ_OK && r.status == OQ_OK)
            check(a.n_dst == r.n_dst && !memcmp(d, full, r.n_dst),
                  "streaming bytes", sl, cut);
        free(d);
    }
    free(full);
}

static void
scan_record(const uint8_t *p0, size_t len)
{
    ++n_records;
    std::vector<uint8_t> rec = dup(p0, len);
    const uint8_t *p = len ? rec.data() : nullptr;
    std::vector<qhuff_literal> lits(len + 1);
    for (int kind = 0; kind < 2; ++kind)
    {
        uint32_t n = 0;
        size_t used = 0;
        const int rc = kind
            ? qhuff_scan_encoder_stream(p, len, 0, lits.data(),
                                        (uint32_t) lits.size(), &n, &used)
            : qhuff_scan_field_section(p, len, 0, lits.data(),
                                       (uint32_t) lits.size(), &n);
        check(rc == QHUFF_OK || rc == QHUFF_ETRUNC || rc == QHUFF_EPROTO,
              "scan rc", kind, (unsigned) -rc);
        if (rc != QHUFF_OK)
            continue;
        check(!kind || used <= len, "consumed", kind, (unsigned) used);
        // a short literal array: ERANGE, never a write past it
        if (n > 1)
        {
            std::vector<qhuff_literal> few(1);
            uint32_t m = 0;
            const int r2 = kind
                ? qhuff_scan_encoder_stream(p, len, 0, few.data(), 1, &m, &used)
                : qhuff_scan_field_section(p, len, 0, few.data(), 1, &m);
            check(r2 == QHUFF_ERANGE && m == n, "erange", kind, n);
        }
        for (uint32_t i = 0; i < n; ++i)
        {
            const qhuff_literal &l = lits[i];
            ++n_lits;
            check((uint64_t) l.pos + l.len <= len && l.hdr_len >= 1
                  && l.hdr_len <= l.pos && l.instr < l.pos, "span", i, l.pos);
            if ((uint64_t) l.pos + l.len > len)
                continue;
            if (l.huffman)
                check_huffman(p + l.pos, l.len);
        }
    }
}

static void
havoc(const uint8_t *p, size_t len, int rounds)
{
    for (int r = 0; r < rounds; ++r)
    {
        std::vector<uint8_t> b(p, p + len);
        const int ops = 1 + (int) (rnd() % 3);
        for (int k = 0; k < ops && !b.empty(); ++k)
        {
            const size_t j = rnd() % b.size();
            switch (rnd() % 4)
            {
            case 0: b[j] ^= (uint8_t) (1u << (rnd() % 8)); break;
            case 1: b[j] = (uint8_t) rnd(); break;
            case 2: b.resize(j); break;
            default:
                b.insert(b.begin() + (long) j, 1 + rnd() % 8, (uint8_t) rnd());
            }
        }
        scan_record(b.data(), b.size());
    }
}

int
main(int argc, char **argv)
{
    oq_init();
    for (unsigned s = 0; s < 256; ++s)
    {
        uint32_t c;
        unsigned b;
        oq_code_of(s, &c, &b);
        code_len[s] = (uint8_t) b;
    }
    for (int a = 1; a < argc; ++a)
    {
        FILE *f = fopen(argv[a], "rb");
        if (!f)
            return perror(argv[a]), 2;
        std::vector<uint8_t> data;
        uint8_t tmp[4096];
        size_t k;
        while ((k = fread(tmp, 1, sizeof tmp, f)) > 0)
            data.insert(data.end(), tmp, tmp + k);
        fclose(f);
        size_t pos = 0;
        while (pos + 12 < data.size())
        {
            uint64_t sid = 0;
            uint32_t size = 0;
            for (int i = 0; i < 8; ++i)
                sid = sid << 8 | data[pos + i];
            for (int i = 8; i < 12; ++i)
                size = size << 8 | data[pos + i];
            pos += 12;
            if (size > data.size() - pos)
                size = (uint32_t) (data.size() - pos);
            (void) sid;
            scan_record(data.data() + pos, size);
            havoc(data.data() + pos, size, 4);
            pos += size;
        }
    }
    for (int i = 0; i < 4000; ++i)
    {
        uint8_t b[64];
        const size_t n = rnd() % sizeof b;
        for (size_t j = 0; j < n; ++j)
            b[j] = (uint8_t) rnd();
        scan_record(b, n);
        check_huffman(b, (uint32_t) n);
    }
    printf("records %lu literals %lu huffman %lu checks %lu failures %lu\n",
           n_records, n_lits, n_huff, n_checks, n_bad);
    return n_bad ? 1 : 0;
}
