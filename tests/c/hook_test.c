/*
 * hook_test.c -- examples/qhuff_hook.c (the INTEGRATION.md seams) against
 * the CPU oracle (TEST INFRASTRUCTURE: links oracle/_build/libqhuff_oracle.so
 * as the checker only).
 *
 *   hook_test enc FILE.qif...          one memo batch per file (every name
 *       and value), then for every string, prefix 3/5/7, two dst[0] values
 *       and dst_len around the need: lsqpack_qhuff_enc_lookup ==
 *       oq_enc_enc_str (lsqpack_enc_enc_str), lsqpack_qhuff_enc_str_size ==
 *       oq_enc_str_size (qenc_enc_str_size); moved or edited strings miss.
 *   hook_test dec FILE.out.256.100.1...   one memo batch per interop file
 *       (every literal of every frame), then for every Huffman literal and
 *       dst_len around its decoded length: the seam (lookup, else the
 *       reference decoder, as patched lsqpack_huff_decode runs) ==
 *       oq_huff_decode (lsqpack_huff_decode) in status, n_dst, n_src and
 *       bytes.
 * Prints counts; exit 0 only with no mismatch and hits > 0.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qhuff_hook.h"

/* oracle (lsqpack.c restatement, oracle/qhuff_oracle.c) */
struct oq_retval { int status; unsigned n_dst, n_src; };
struct oq_dec_state { int resume; uint8_t state, eos; };
unsigned oq_enc_str_size(const unsigned char *str, unsigned len);
int oq_enc_enc_str(unsigned prefix_bits, unsigned char *dst, size_t dst_len,
                   const unsigned char *str, unsigned str_len);
struct oq_retval oq_huff_decode(const unsigned char *src, int src_len,
                                unsigned char *dst, int dst_len,
                                struct oq_dec_state *st, int final);

static uint8_t *
slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(n > 0 ? (size_t) n + 1 : 1);
    if (b && fread(b, 1, (size_t) n, f) != (size_t) n)
    {
        free(b);
        b = NULL;
    }
    fclose(f);
    *len = (size_t) n;
    return b;
}

static unsigned long hits, misses, checks, bad;

static void
check(int ok, const char *what, unsigned i, unsigned a)
{
    ++checks;
    if (!ok && bad++ < 10)
        fprintf(stderr, "mismatch: %s string %u arg %u\n", what, i, a);
}

/* names and values of a QIF file, in place (qif: name TAB value lines,
 * blank line between header lists, '#' comments) */
static unsigned
qif_strings(uint8_t *b, size_t len, const unsigned char **strs,
            unsigned *lens, unsigned cap)
{
    unsigned n = 0;
    size_t p = 0;
    while (p < len && n + 2 <= cap)
    {
        size_t e = p;
        while (e < len && b[e] != '\n')
            ++e;
        if (e > p && b[p] != '#')
        {
            size_t t = p;
            while (t < e && b[t] != '\t')
                ++t;
            if (t < e)
            {
                strs[n] = b + p;
                lens[n++] = (unsigned) (t - p);
                strs[n] = b + t + 1;
                lens[n++] = (unsigned) (e - t - 1);
            }
        }
        p = e + 1;
    }
    return n;
}

static int
run_enc(struct qhuff_memo *m, const char *path)
{
    size_t len;
    uint8_t *b = slurp(path, &len);
    if (!b)
        return perror(path), 1;
    const unsigned cap = 1u << 20;
    const unsigned char **strs = malloc(cap * sizeof *strs);
    unsigned *lens = malloc(cap * sizeof *lens);
    const unsigned n = qif_strings(b, len, strs, lens, cap);
    int rc = qhuff_memo_encode(m, strs, lens, n);
    if (rc != QHUFF_OK)
        return fprintf(stderr, "memo_encode %d\n", rc), 1;
    static unsigned char got[1 << 17], want[1 << 17];
    for (unsigned i = 0; i < n; ++i)
    {
        const int sz = lsqpack_qhuff_enc_str_size(strs[i], lens[i]);
        check(sz >= 0 && (unsigned) sz == oq_enc_str_size(strs[i], lens[i]),
              "enc_str_size", i, 0);
        for (unsigned p = 3; p <= 7; p += 2)
            for (unsigned f = 0; f < 2; ++f)
            {
                const unsigned char first =
                    f ? (unsigned char) (0xffu << (p + 1)) : 0;
                want[0] = first;
                const int need = oq_enc_enc_str(p, want, sizeof want,
                                                strs[i], lens[i]);
                const size_t dls[] = {0, 1, 2, (size_t) need - 1,
                                      (size_t) need, (size_t) need + 7};
                for (unsigned k = 0; k < sizeof dls / sizeof dls[0]; ++k)
                {
                    const size_t dl = dls[k];
                    if (dl > sizeof got)
                        continue;
                    got[0] = want[0] = first;
                    const int r = lsqpack_qhuff_enc_lookup(p, got, dl,
                                                           strs[i], lens[i]);
                    const int w = oq_enc_enc_str(p, want, dl, strs[i],
                                                 lens[i]);
                    if (r == LSQPACK_QHUFF_MISS)
                        ++misses;
                    else
                        ++hits;
                    check(r == w && (w < 0 || memcmp(got, want, w) == 0),
                          "enc_enc_str", i, (unsigned) dl);
                }
            }
    }
    /* a copy at another address, and an edited string, must miss */
    if (n)
    {
        unsigned char *copy = malloc(lens[0] + 1);
        memcpy(copy, strs[0], lens[0]);
        check(lsqpack_qhuff_enc_lookup(3, got, sizeof got, copy, lens[0])
              == LSQPACK_QHUFF_MISS, "moved string misses", 0, 0);
        if (lens[0])
        {
            unsigned char *s = (unsigned char *) strs[0];
            s[0] ^= 1;
            check(lsqpack_qhuff_enc_lookup(3, got, sizeof got, s, lens[0])
                  == LSQPACK_QHUFF_MISS, "edited string misses", 0, 0);
            s[0] ^= 1;
        }
        free(copy);
    }
    printf("enc %s: strings %u\n", path, n);
    free(strs);
    free(lens);
    free(b);
    return 0;
}

static uint64_t
be(const uint8_t *p, int n)
{
    uint64_t v = 0;
    for (int i = 0; i < n; ++i)
        v = v << 8 | p[i];
    return v;
}

static int
run_dec(struct qhuff_memo *m, const char *path)
{
    size_t len;
    uint8_t *buf = slurp(path, &len);
    if (!buf)
        return perror(path), 1;
    uint32_t cap = 1u << 16, n = 0, k;
    struct qhuff_literal *lits = malloc(cap * sizeof *lits);
    size_t pos = 0;
    while (pos + 12 <= len)     /* bin/interop-encode.c:120-170 framing */
    {
        const uint64_t sid = be(buf + pos, 8);
        const uint32_t flen = (uint32_t) be(buf + pos + 8, 4);
        if (pos + 12 + flen > len)
            break;
        int rc;
        k = 0;
        if (sid == 0)
        {
            size_t used;
            rc = qhuff_scan_encoder_stream(buf + pos + 12, flen,
                                           (uint32_t) (pos + 12), lits + n,
                                           cap - n, &k, &used);
        }
        else
        {
            rc = qhuff_scan_field_section(buf + pos + 12, flen,
                                          (uint32_t) (pos + 12), lits + n,
                                          cap - n, &k);
            if (rc == QHUFF_ETRUNC)
                rc = QHUFF_OK, k = 0;
        }
        if (rc != QHUFF_OK)
            return fprintf(stderr, "scan %d\n", rc), 1;
        n += k;
        pos += 12 + flen;
    }
    int rc = qhuff_memo_decode(m, buf, lits, n);
    if (rc != QHUFF_OK)
        return fprintf(stderr, "memo_decode %d\n", rc), 1;
    static unsigned char got[1 << 17], want[1 << 17];
    unsigned n_huff = 0;
    for (uint32_t i = 0; i < n; ++i)
    {
        if (!lits[i].huffman)
            continue;
        ++n_huff;
        const unsigned char *src = buf + lits[i].pos;
        const int sl = (int) lits[i].len;
        struct oq_dec_state st0 = {0, 0, 0};
        const struct oq_retval full = oq_huff_decode(src, sl, want,
                                                     sizeof want, &st0, 1);
        const int nd = (int) full.n_dst;
        const int dls[] = {0, nd - 1, nd, nd + 1, sl + sl / 2, 2 * sl + 8};
        for (unsigned j = 0; j < sizeof dls / sizeof dls[0]; ++j)
        {
            const int dl = dls[j];
            if (dl < 0)
                continue;
            struct oq_dec_state a = {0, 0, 0}, b = {0, 0, 0};
            struct qhuff_decode_retval rv;
            struct oq_retval g;
            if (lsqpack_qhuff_dec_lookup(src, sl, got, dl, &rv))
            {
                ++hits;
                g.status = (int) rv.status;
                g.n_dst = rv.n_dst;
                g.n_src = rv.n_src;
            }
            else
            {
                ++misses;
                g = oq_huff_decode(src, sl, got, dl, &a, 1);
            }
            const struct oq_retval w = oq_huff_decode(src, sl, want, dl, &b,
                                                      1);
            check(g.status == w.status && g.n_dst == w.n_dst
                  && g.n_src == w.n_src && memcmp(got, want, w.n_dst) == 0,
                  "huff_decode", i, (unsigned) dl);
        }
    }
    /* a receive buffer reused at the same address: once the
     * bytes under a memoised payload change, the lookup must miss */
    for (uint32_t i = 0; i < n; ++i)
        if (lits[i].huffman && lits[i].len)
        {
            unsigned char *p = buf + lits[i].pos;
            const int sl = (int) lits[i].len;
            const unsigned char keep = p[0];
            struct qhuff_decode_retval rv;
            const int before = lsqpack_qhuff_dec_lookup(p, sl, got, sizeof got,
                                                        &rv);
            p[0] ^= 0x5a;
            check(!lsqpack_qhuff_dec_lookup(p, sl, got, sizeof got, &rv),
                  "stale payload hit", i, 0);
            p[0] = keep;
            check(lsqpack_qhuff_dec_lookup(p, sl, got, sizeof got, &rv)
                  == before, "restored payload", i, 0);
        }
    printf("dec %s: literals %u (huffman %u)\n", path, n, n_huff);
    free(lits);
    free(buf);
    return 0;
}

int
main(int argc, char **argv)
{
    if (argc < 3 || (strcmp(argv[1], "enc") && strcmp(argv[1], "dec")))
        return fprintf(stderr, "usage: %s enc|dec FILE...\n", argv[0]), 2;
    qhuff_ctx *ctx;
    int rc = qhuff_open(0, &ctx);
    if (rc != QHUFF_OK)
        return fprintf(stderr, "qhuff_open %d\n", rc), 1;
    struct qhuff_memo *m = qhuff_memo_new(ctx);
    lsqpack_qhuff_use(m);
    for (int a = 2; a < argc; ++a)
        if ((argv[1][0] == 'e' ? run_enc : run_dec)(m, argv[a]))
            return 1;
    printf("checks %lu hits %lu misses %lu mismatches %lu\n", checks, hits,
           misses, bad);
    qhuff_memo_free(m);
    qhuff_close(ctx);
    return (bad || !hits) ? 1 : 0;
}
