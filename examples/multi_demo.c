/*
 * multi_demo.c -- one header-string batch over several GPUs from plain C99
 * (include/qhuff.h ABI 7, qhuff_*_batch_host_multi): the call cuts the batch
 * by bytes into one shard per context, runs every shard on its own host
 * thread and GPU, and returns one output with global offsets -- what a
 * server behind lsqpack.h that gathers literals from many connections
 * would call once per batch.  Checks the result against a single-context
 * call and the round trip.
 *
 * usage: multi_demo [CONTEXTS [STRINGS]]   (contexts spread over the
 * visible devices round-robin; default one per device, 262144 strings)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "qhuff.h"

static int
count_devices(void)
{
    /* qhuff_open fails with QHUFF_ENODEV past the last device */
    int n = 0;
    for (;; ++n)
    {
        qhuff_ctx *c = NULL;
        if (qhuff_open(n, &c) != QHUFF_OK)
            break;
        qhuff_close(c);
    }
    return n;
}

int
main(int argc, char **argv)
{
    const int ndev = count_devices();
    if (ndev < 1)
    {
        fprintf(stderr, "no device: %s\n", qhuff_last_error(NULL));
        return 2;
    }
    const uint32_t g = argc > 1 ? (uint32_t) atoi(argv[1]) : (uint32_t) ndev;
    const uint32_t n = argc > 2 ? (uint32_t) atoi(argv[2]) : 262144u;
    if (g < 1 || g > 64)
        return 2;
    qhuff_ctx *ctx[64];
    for (uint32_t k = 0; k < g; ++k)
        if (qhuff_open((int) (k % (uint32_t) ndev), &ctx[k]) != QHUFF_OK)
        {
            fprintf(stderr, "qhuff_open: %s\n", qhuff_last_error(NULL));
            return 2;
        }
    static const uint8_t alpha[] = "abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, ";
    uint8_t *data = malloc((size_t) n * 64 + 1);
    uint32_t *off = malloc(4 * ((size_t) n + 1));
    const uint64_t raw = qhuff_synth_batch(7, n, 8, 64, alpha,
                                           sizeof(alpha) - 1, data, off);
    const uint64_t eb = qhuff_encode_bound(raw, n, QHUFF_ENC_PAYLOAD);
    uint8_t *enc = malloc(eb), *enc1 = malloc(eb);
    uint32_t *eoff = malloc(4 * ((size_t) n + 1)), *eoff1 = malloc(4 * ((size_t) n + 1));
    int rc = qhuff_encode_batch_host_multi(ctx, g, data, off, n,
                                           QHUFF_ENC_PAYLOAD, enc, eoff);
    int rc1 = qhuff_encode_batch_host(ctx[0], data, off, n, QHUFF_ENC_PAYLOAD,
                                      enc1, eoff1);
    if (rc || rc1)
    {
        fprintf(stderr, "encode: %d / %d\n", rc, rc1);
        return 1;
    }
    const uint32_t hb = eoff[n];
    long bad = memcmp(eoff, eoff1, 4 * ((size_t) n + 1)) != 0
             || memcmp(enc, enc1, hb) != 0;
    const uint64_t db = qhuff_decode_bound(hb, n);
    uint8_t *dec = malloc(db), *st = malloc(n);
    uint32_t *doff = malloc(4 * ((size_t) n + 1));
    rc = qhuff_decode_batch_host_multi(ctx, g, enc, eoff, n, dec, doff, st);
    if (rc)
    {
        fprintf(stderr, "decode: %d\n", rc);
        return 1;
    }
    for (uint32_t i = 0; i < n; ++i)
        bad += st[i] != QHUFF_DEC_OK;
    bad += memcmp(doff, off, 4 * ((size_t) n + 1)) != 0
         || memcmp(dec, data, raw) != 0;
    /* the same calls again on registered buffers (qhuff_host_register):
     * DMA straight from / into them, the same results */
    uint8_t *dec2 = malloc(db), *st2 = malloc(n);
    uint32_t *doff2 = malloc(4 * ((size_t) n + 1));
    void *reg[] = {data, off, enc1, eoff1, dec2, doff2, st2};
    const size_t regb[] = {raw ? raw : 1, 4 * ((size_t) n + 1), eb,
                           4 * ((size_t) n + 1), db, 4 * ((size_t) n + 1), n};
    for (int k = 0; k < 7; ++k)
        if (qhuff_host_register(reg[k], regb[k]) != QHUFF_OK)
        {
            fprintf(stderr, "qhuff_host_register: %s\n", qhuff_last_error(NULL));
            return 1;
        }
    rc = qhuff_encode_batch_host_multi(ctx, g, data, off, n, QHUFF_ENC_PAYLOAD,
                                       enc1, eoff1);
    rc1 = qhuff_decode_batch_host_multi(ctx, g, enc1, eoff1, n, dec2, doff2, st2);
    for (int k = 0; k < 7; ++k)
        qhuff_host_unregister(reg[k]);
    if (rc || rc1)
    {
        fprintf(stderr, "registered: %d / %d\n", rc, rc1);
        return 1;
    }
    bad += memcmp(eoff1, eoff, 4 * ((size_t) n + 1)) != 0
         || memcmp(enc1, enc, hb) != 0 || memcmp(doff2, doff, 4 * ((size_t) n + 1)) != 0
         || memcmp(dec2, dec, raw) != 0 || memcmp(st2, st, n) != 0;
    printf("multi_demo: %u contexts on %d device(s), %u strings, %llu raw / "
           "%u Huffman bytes, mismatches %ld (staged and registered)\n", g,
           ndev, n, (unsigned long long) raw, hb, bad);
    for (uint32_t k = 0; k < g; ++k)
        qhuff_close(ctx[k]);
    free(data); free(off); free(enc); free(enc1); free(eoff); free(eoff1);
    free(dec); free(st); free(doff); free(dec2); free(st2); free(doff2);
    return bad ? 1 : 0;
}
