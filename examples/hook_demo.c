/*
 * hook_demo.c -- the drop-in seams of INTEGRATION.md section 2, exercised
 * from plain C99 against include/qhuff.h + libqhuff.so only.
 *
 * Input: an offline-interop file written by the reference's
 * bin/interop-encode (bin/interop-encode.c:120-170: u64 BE stream id, u32 BE
 * length, payload; stream 0 = encoder stream), e.g.
 * tests/golden/data/netbsd.out.256.100.1.
 *
 *  1. decoder side: every field section / encoder-stream chunk is scanned
 *     for string literals (qhuff_scan_field_section / _encoder_stream) and
 *     ALL literals of the file are decoded in one GPU batch
 *     (qhuff_decode_literals_host);
 *  2. encoder side: the decoded strings are Huffman-coded in one GPU batch
 *     (qhuff_encode_batch_host, QHUFF_ENC_PAYLOAD) and every literal is
 *     re-framed with qhuff_frame_literal (= lsqpack_enc_enc_str) using the
 *     wire literal's own first byte -- which must give back the reference's
 *     bytes exactly;
 *
 * Exit status 0 only if every literal round-trips byte for byte.
 * Build: make -C examples  (gcc, links ../ls-qpack_amd/libqhuff.so)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qhuff.h"

static uint8_t *
slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *b = malloc(n > 0 ? (size_t) n : 1);
    if (b && fread(b, 1, (size_t) n, f) != (size_t) n)
    {
        free(b);
        b = NULL;
    }
    fclose(f);
    *len = (size_t) n;
    return b;
}

static uint64_t
be(const uint8_t *p, int n)
{
    uint64_t v = 0;
    for (int i = 0; i < n; ++i)
        v = v << 8 | p[i];
    return v;
}

int
main(int argc, char **argv)
{
    if (argc < 2)
    {
        fprintf(stderr, "usage: %s INTEROP_FILE\n", argv[0]);
        return 2;
    }
    size_t len;
    uint8_t *buf = slurp(argv[1], &len);
    if (!buf)
    {
        perror(argv[1]);
        return 2;
    }
    qhuff_ctx *ctx;
    int rc = qhuff_open(0, &ctx);
    if (rc != QHUFF_OK)
    {
        fprintf(stderr, "qhuff_open: %d\n", rc);
        return 1;
    }

    /* 1. scan every frame; literal positions are relative to buf */
    uint32_t cap = 1u << 16, n = 0;
    struct qhuff_literal *lits = malloc(cap * sizeof *lits);
    size_t pos = 0;
    while (pos + 12 <= len)
    {
        const uint64_t sid = be(buf + pos, 8);
        const uint32_t flen = (uint32_t) be(buf + pos + 8, 4);
        if (pos + 12 + flen > len)
            break;                                   /* truncated file */
        const uint8_t *fr = buf + pos + 12;
        uint32_t k = 0;
        if (sid == 0)
        {
            size_t used;
            rc = qhuff_scan_encoder_stream(fr, flen, (uint32_t) (pos + 12),
                                           lits + n, cap - n, &k, &used);
        }
        else
        {
            rc = qhuff_scan_field_section(fr, flen, (uint32_t) (pos + 12),
                                          lits + n, cap - n, &k);
            if (rc == QHUFF_ETRUNC)
                rc = QHUFF_OK, k = 0;
        }
        if (rc != QHUFF_OK)
        {
            fprintf(stderr, "scan at %zu: %d\n", pos, rc);
            return 1;
        }
        n += k;
        pos += 12 + flen;
    }

    uint8_t *dec = malloc(qhuff_literals_bound(lits, n));
    uint32_t *dec_off = malloc((n + 1) * sizeof *dec_off);
    uint8_t *st = malloc(n ? n : 1);
    rc = qhuff_decode_literals_host(ctx, buf, lits, n, dec, dec_off, st);
    if (rc != QHUFF_OK)
    {
        fprintf(stderr, "decode_literals: %d (%s)\n", rc, qhuff_last_error(ctx));
        return 1;
    }
    uint32_t n_huff = 0, bad = 0;
    for (uint32_t i = 0; i < n; ++i)
    {
        n_huff += lits[i].huffman;
        bad += st[i] != QHUFF_DEC_OK;
    }

    /* 2. one PAYLOAD batch for all decoded strings, then frame each */
    const uint64_t eb = qhuff_encode_bound(dec_off[n], n, QHUFF_ENC_PAYLOAD);
    uint8_t *huf = malloc(eb);
    uint32_t *huf_off = malloc((n + 1) * sizeof *huf_off);
    rc = qhuff_encode_batch_host(ctx, dec, dec_off, n, QHUFF_ENC_PAYLOAD, huf,
                                 huf_off);
    if (rc != QHUFF_OK)
    {
        fprintf(stderr, "encode_batch_host: %d\n", rc);
        return 1;
    }
    uint32_t mismatch = 0;
    unsigned char frame[1 << 16];
    for (uint32_t i = 0; i < n; ++i)
    {
        const uint32_t start = lits[i].pos - lits[i].hdr_len;
        frame[0] = buf[start];
        const int r = qhuff_frame_literal(lits[i].prefix_bits, frame,
                                          sizeof frame, dec + dec_off[i],
                                          dec_off[i + 1] - dec_off[i],
                                          huf + huf_off[i],
                                          huf_off[i + 1] - huf_off[i]);
        const uint32_t wire = lits[i].pos + lits[i].len - start;
        if (r < 0 || (uint32_t) r != wire || memcmp(frame, buf + start, wire))
            ++mismatch;
    }

    printf("literals %u (huffman %u), decode errors %u, re-framed mismatches "
           "%u\n", n, n_huff, bad, mismatch);
    qhuff_close(ctx);
    return (bad || mismatch || n == 0) ? 1 : 0;
}
